set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tracking.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_trk.log 2>&1 || { tail -40 gpurun_out/t_trk.log; exit 1; }
tail -2 gpurun_out/t_trk.log
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --no-ba --no-pose --no-cpu-baseline --pipelined-streams 0 --no-all-cores > gpurun_out/b_trk.json 2> gpurun_out/b_trk.err
