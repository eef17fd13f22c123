set -eo pipefail
export TMPDIR=/tmp
# scratch GPU step (development): ORB parity tests + forced-gate kernel timings of abl/ variants
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_orb.py > gpurun_out/pytest.log 2>&1
