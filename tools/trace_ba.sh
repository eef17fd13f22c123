#!/bin/bash
# Kernel + copy trace of the BA ablation driver (development tool): per-iteration timeline of
# the LM kernels, their gaps and the host round trips.  On the GPU box:
#   bash tools/trace_ba.sh            -> gpurun_out/batrace/ (gzip'd CSVs)
# here:  python tools/trace_gaps.py gpurun_out/batrace
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/batrace
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/batrace/t -o run --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-pose --no-tracking --no-cpu-baseline --no-all-cores \
    --pipelined-streams 0 --profile 0 > gpurun_out/batrace/out.log 2>&1
find gpurun_out/batrace -name '*.csv' -exec gzip -f {} \;
