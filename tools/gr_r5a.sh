# Round 5, first GPU call: VALU issue probe + SQ issue/stall counters of the ORB-only bench.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/valu_probe > gpurun_out/valu_probe.txt 2>&1
cat gpurun_out/valu_probe.txt
bash tools/pmc_sq.sh
echo done
