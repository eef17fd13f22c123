# dev: variant timings (tools/abl.py) then the SQ counter pass of the ORB-only bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/abl.py run "$1" > gpurun_out/abl_run.log 2>&1 && bash tools/gr_pmc_sq.sh
