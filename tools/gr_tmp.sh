set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_orb.py > gpurun_out/pytest.log 2>&1
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-ba --no-pose --no-tracking --no-cpu-baseline --pipelined-streams 0 --no-all-cores --orb-variant rbrief31 > gpurun_out/b31.json 2> gpurun_out/b31.err
