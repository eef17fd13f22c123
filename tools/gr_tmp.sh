set -eo pipefail
export TMPDIR=/tmp
MAGE_ABLATE_GATE=89 timeout -k 10 300 python3 tools/abl.py run gprev,gnu,gprev,gnu,gprev,gnu > gpurun_out/abl.log 2>&1
