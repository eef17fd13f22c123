set -eo pipefail
export TMPDIR=/tmp
# scratch GPU step (development): BA determinism + parity, then variant timings
timeout -k 10 120 python3 -u tools/ba_det_probe.py > gpurun_out/det.log 2>&1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ba.py tests/test_gpu_tracking.py tests/test_local_ba.py > gpurun_out/pytest.log 2>&1
timeout -k 10 300 python3 tools/ablate_ba.py libs head,pe,head,pe,head,pe > gpurun_out/ab_ba.log 2>&1
