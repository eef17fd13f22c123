#!/bin/bash
# Profiling recipe for the committed evidence (run on the GPU box from the repo root):
#   kernel trace + stats, then FETCH_SIZE, WRITE_SIZE and SQ VALU/MFMA counters in separate passes
#   (never combined with trace domains), then the summary into profiles/<tag>_*.
# usage: bash tools/profile_round.sh <tag>
set -eo pipefail
TAG=${1:-r1}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
CMD="python3 bench.py --steps 10 --warmup 3 --ba-iters 20 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $CMD > $OUT/bench_trace.json 2> $OUT/trace.err
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- $CMD > /dev/null 2> $OUT/fetch.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- $CMD > /dev/null 2> $OUT/write.err
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES -d $OUT/pmc_valu -o run --output-format csv -- $CMD > /dev/null 2> $OUT/valu.err
python3 tools/rocprof_summary.py $OUT $TAG > $OUT/summary.md
cp $OUT/trace/run_kernel_stats.csv profiles/${TAG}_kernel_stats.csv
timeout -k 10 400 python3 bench.py > $OUT/bench_final.json 2> $OUT/bench_final.err
