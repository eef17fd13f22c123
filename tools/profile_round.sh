#!/bin/bash
# Profiling recipe for the committed evidence (run on the GPU box from the repo root):
#   kernel trace + stats, then FETCH_SIZE, WRITE_SIZE and SQ VALU/MFMA counters in separate passes
#   (never combined with trace domains), for bench.py and for tools/bench_rows.py (the §8 rows the
#   headline does not exercise), then the summaries into profiles/<tag>_*.
# usage: bash tools/profile_round.sh <tag> [main|rows]   (on the box; only gpurun_out/ comes back)
#        bash tools/profile_round.sh <tag> collect   (here: summaries from gpurun_out/ into profiles/)
set -eo pipefail
TAG=${1:-r1}
export TMPDIR=/tmp
run_set() {  # <out dir> <command...>
    local OUT=$1; shift
    mkdir -p $OUT
    python3 -c "from mageslam_amd.build import kernel_sources_sha; print(kernel_sources_sha())" > $OUT/sources_sha
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- "$@" > $OUT/trace.json 2> $OUT/trace.err
    timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- "$@" > /dev/null 2> $OUT/fetch.err
    timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- "$@" > /dev/null 2> $OUT/write.err
    timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE -d $OUT/pmc_valu -o run --output-format csv -- "$@" > /dev/null 2> $OUT/valu.err
    # only the stats and counter tables come back (gpurun returns <= 64 MiB of gpurun_out/)
    find $OUT -name '*.csv' ! -name run_kernel_stats.csv ! -name run_counter_collection.csv ! -name run_kernel_trace.csv -delete
    find $OUT \( -name run_counter_collection.csv -o -name run_kernel_trace.csv \) -exec gzip -f {} \;
}
OUT=gpurun_out/prof_$TAG
ORB=gpurun_out/prof_${TAG}_orb
ROWS=gpurun_out/prof_${TAG}_rows
ORB_CMD="python3 bench.py --steps 10 --warmup 3 --no-ba --no-pose --no-tracking --no-cpu-baseline --pipelined-streams 0 --no-all-cores --no-rbrief31"
ORB31=gpurun_out/prof_${TAG}_orb31
ORB31_CMD="python3 bench.py --steps 10 --warmup 3 --no-ba --no-pose --no-tracking --no-cpu-baseline --pipelined-streams 0 --no-all-cores --orb-variant rbrief31"
if [ "$2" = collect ]; then
  if [ -d $OUT/trace ]; then
    python3 tools/rocprof_summary.py $OUT $TAG "python bench.py" 3 > /dev/null
    cp $OUT/trace/run_kernel_stats.csv profiles/${TAG}_kernel_stats.csv
    cp profiles/${TAG}_pmc_summary.json profiles/pmc_summary_ba.json  # BA kernels' counters (bench.py)
  fi
    python3 tools/rocprof_summary.py $ROWS ${TAG}_rows "python tools/bench_rows.py" > /dev/null
    cp profiles/${TAG}_rows_pmc_summary.json profiles/pmc_summary_rows.json  # pose-only BA counters (bench.py)
    cp $ROWS/trace/run_kernel_stats.csv profiles/${TAG}_rows_kernel_stats.csv
    cp $ROWS/trace.json profiles/${TAG}_rows.jsonl
    cp $OUT/bench_final.json profiles/${TAG}_bench.json
    # the headline ORB leg alone (every fast_nms launch is a 256-frame batch, so the average
    # duration is the one bench.py prices the roofline on); its counters become
    # profiles/pmc_summary.json, which bench.py reads for roofline.traffic
    python3 tools/rocprof_summary.py $ORB ${TAG}_orb "${ORB_CMD#python3 }" 3 > /dev/null
    cp $ORB/trace/run_kernel_stats.csv profiles/${TAG}_orb_kernel_stats.csv
    cp $ORB/trace.json profiles/${TAG}_orb_bench.json
    cp profiles/${TAG}_orb_pmc_summary.json profiles/pmc_summary.json
    # the rBRIEF-31 variant (4 levels, patch 31, orientation) alone: profiles/pmc_summary_rbrief31.json
    python3 tools/rocprof_summary.py $ORB31 ${TAG}_orb31 "${ORB31_CMD#python3 }" 3 > /dev/null
    cp $ORB31/trace/run_kernel_stats.csv profiles/${TAG}_orb31_kernel_stats.csv
    cp $ORB31/trace.json profiles/${TAG}_orb31_bench.json
    cp profiles/${TAG}_orb31_pmc_summary.json profiles/pmc_summary_rbrief31.json
    exit 0
fi
# optional phase (one gpurun call each when the whole round would not fit one call's limit):
#   main = headline + ORB-only sets, rows = the per-row set + the final default bench line
PHASE=${2:-all}
if [ "$PHASE" = all ] || [ "$PHASE" = main ]; then
    run_set $OUT python3 bench.py --steps 10 --warmup 3 --ba-iters 20 --no-cpu-baseline --pipelined-streams 0 --no-all-cores --no-tracking --no-rbrief31
    run_set $ORB $ORB_CMD
    run_set $ORB31 $ORB31_CMD
fi
if [ "$PHASE" = orb ]; then  # the ORB-only and rBRIEF-31 sets alone (when only orb.hip changed)
    run_set $ORB $ORB_CMD
    run_set $ORB31 $ORB31_CMD
fi
if [ "$PHASE" = all ] || [ "$PHASE" = rows ]; then
    run_set $ROWS python3 tools/bench_rows.py
    mkdir -p $OUT
    timeout -k 10 600 python3 bench.py > $OUT/bench_final.json 2> $OUT/bench_final.err
fi
