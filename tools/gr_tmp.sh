set -eo pipefail
export TMPDIR=/tmp
# scratch GPU step (development): matcher parity, then the ORB-only bench
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_match.py tests/test_gpu_bow.py > gpurun_out/pytest.log 2>&1
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 3 --no-ba --no-pose --no-tracking --no-cpu-baseline --no-rbrief31 > gpurun_out/b_orb.json 2> gpurun_out/b_orb.err
