# FAST ablation variants under the VALU counters (dev): MAGE_ABLATE_GATE forced
set -eo pipefail
export TMPDIR=/tmp
export MAGE_ABLATE_GATE=${1:-83}
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU -d gpurun_out/abl_pmc -o run --output-format csv -- python3 tools/ablate_fast.py run ${2:-0,1,17,35,39,47} > gpurun_out/abl_pmc.log 2>&1
find gpurun_out/abl_pmc -name '*.csv' ! -name run_counter_collection.csv -delete
timeout -k 10 200 python3 tools/ablate_fast.py run ${2:-0,1,17,35,39,47} > gpurun_out/abl_time.log 2>&1
