set -eo pipefail
export TMPDIR=/tmp
# scratch GPU step (development): BA parity incl. rejected trials
timeout -k 10 400 python3 -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ba.py > gpurun_out/pytest.log 2>&1
