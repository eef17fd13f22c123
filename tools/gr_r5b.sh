# Round 5: FAST ablation timings + per-variant SQ instruction counts + ORB parity of the default build.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
V=${1:-base,d16,nob,noex,nonms,noscore,noload}
export MAGE_ABLATE_GATE=${GATE:-89}
timeout -k 10 300 python3 tools/abl.py run $V > gpurun_out/abl_run.log 2>&1
cat gpurun_out/abl_run.log
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE -d gpurun_out/abl_pmc -o run --output-format csv -- python3 tools/abl.py run $V > gpurun_out/abl_pmc.log 2>&1
find gpurun_out/abl_pmc -name '*.csv' ! -name run_counter_collection.csv -delete
if [ -n "$PYTEST" ]; then
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread $PYTEST > gpurun_out/pytest.log 2>&1; tail -5 gpurun_out/pytest.log
fi
echo done
