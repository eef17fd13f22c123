# round-4 batch d: pose-BA observations staged in LDS — BA / tracking parity, tracking kernel times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ba.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_ba.log 2>&1 || { tail -40 gpurun_out/t_ba.log; exit 1; }
tail -2 gpurun_out/t_ba.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_tracking.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_trk.log 2>&1 || { tail -40 gpurun_out/t_trk.log; exit 1; }
tail -2 gpurun_out/t_trk.log
timeout -k 10 200 python3 -u tools/track_kernels.py 240 > gpurun_out/track_kernels.json 2> gpurun_out/track_kernels.err || exit 1
echo all-done
