set -eo pipefail
export TMPDIR=/tmp
# scratch GPU step (development): variant timings, alternating
timeout -k 10 300 python3 tools/abl.py run head,xorreg,head,xorreg,head,xorreg,head,xorreg,head,xorreg > gpurun_out/abl_run.log 2>&1
