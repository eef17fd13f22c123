# rBRIEF-31 leg: kernel trace + SQ counters (dev), one pass each
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
CMD="python3 bench.py --steps 10 --warmup 3 --no-ba --no-pose --no-tracking --no-cpu-baseline --pipelined-streams 0 --no-all-cores --orb-variant rbrief31"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr31 -o run --output-format csv -- $CMD > gpurun_out/tr31.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM -d gpurun_out/pmc31 -o run --output-format csv -- $CMD > gpurun_out/pmc31.log 2>&1
find gpurun_out/tr31 gpurun_out/pmc31 -name '*.csv' ! -name run_counter_collection.csv ! -name run_kernel_stats.csv -delete
