set -eo pipefail
export TMPDIR=/tmp
# scratch GPU step (development): BA determinism + parity, then the BA leg with / without the speculative linearisation
timeout -k 10 120 python3 -u tools/ba_det_probe.py > gpurun_out/det.log 2>&1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ba.py tests/test_gpu_tracking.py tests/test_local_ba.py > gpurun_out/pytest.log 2>&1
timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 2 --no-pose --no-tracking --no-cpu-baseline --no-rbrief31 --pipelined-streams 0 > gpurun_out/b_ba.json 2> gpurun_out/b_ba.err
MAGE_BA_SPEC_LIN=0 timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 2 --no-pose --no-tracking --no-cpu-baseline --no-rbrief31 --pipelined-streams 0 > gpurun_out/b_ba0.json 2> gpurun_out/b_ba0.err
