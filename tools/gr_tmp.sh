set -eo pipefail
export TMPDIR=/tmp
# scratch GPU step (development): BA variant timings
timeout -k 10 300 python3 tools/ablate_ba.py libs head,w4,head,w4,head,w4 > gpurun_out/ab_ba.log 2>&1
