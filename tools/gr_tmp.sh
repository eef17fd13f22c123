set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_orb.py tests/test_gpu_tracking.py > gpurun_out/pytest.log 2>&1
timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-rbrief31 --no-all-cores > gpurun_out/bench_t.json 2> gpurun_out/bench_t.err
