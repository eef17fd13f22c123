set -eo pipefail
export TMPDIR=/tmp
# scratch GPU step (development): parity of the sort users, then variant timings
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_orb.py tests/test_gpu_match.py tests/test_gpu_bow.py tests/test_gpu_tracking.py > gpurun_out/pytest.log 2>&1
timeout -k 10 300 python3 tools/abl.py run head,sortu,head,sortu > gpurun_out/abl_run.log 2>&1
