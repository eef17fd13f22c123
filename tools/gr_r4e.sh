# round-4 batch e: orientation XCD grid + 2 keypoints per wave for wide describe windows — ORB parity, ORB legs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_image.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_orb.log 2>&1 || { tail -40 gpurun_out/t_orb.log; exit 1; }
tail -2 gpurun_out/t_orb.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-ba --no-pose --no-tracking --no-cpu-baseline --no-all-cores --pipelined-streams 0 > gpurun_out/b_orb.json 2> gpurun_out/b_orb.err || { tail -20 gpurun_out/b_orb.err; exit 1; }
echo all-done
