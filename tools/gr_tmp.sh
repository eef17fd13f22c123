set -eo pipefail
export TMPDIR=/tmp
export MAGE_ABLATE_GATE=89
true
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/pytest.log 2>&1
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-ba --no-pose --no-tracking --no-cpu-baseline --pipelined-streams 0 --no-all-cores --orb-variant rbrief31 > gpurun_out/b31.json 2> gpurun_out/b31.err
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-pose --no-tracking --no-cpu-baseline --no-all-cores --no-rbrief31 --pipelined-streams 0 > gpurun_out/bba.json 2> gpurun_out/bba.err
