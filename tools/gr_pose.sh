# pose-only BA: phase stamps of the variant builds, then the pose and tracking parity tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/pose_stamps.py run ${POSE_VARIANTS:-pose} > gpurun_out/pose_stamps3.log 2>&1 || { tail -30 gpurun_out/pose_stamps3.log; exit 1; }
grep -E "^==|E =|->" gpurun_out/pose_stamps3.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ba.py -k "pose" > gpurun_out/t_pose.log 2>&1 || { tail -30 gpurun_out/t_pose.log; exit 1; }
tail -2 gpurun_out/t_pose.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tracking.py > gpurun_out/t_trk.log 2>&1 || { tail -30 gpurun_out/t_trk.log; exit 1; }
tail -2 gpurun_out/t_trk.log
timeout -k 10 300 python -u tools/track_kernels.py 240 > gpurun_out/track_kernels.json 2> gpurun_out/track_kernels.err || { tail -20 gpurun_out/track_kernels.err; exit 1; }
echo all-done
