set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_orb.py > gpurun_out/pytest.log 2>&1
MAGE_ABLATE_GATE=89 timeout -k 10 300 python3 tools/abl.py run sprev,scur,sc,sr,sprev,scur,sc,sr,sprev,scur > gpurun_out/abl.log 2>&1
