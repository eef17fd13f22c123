set -eo pipefail
export TMPDIR=/tmp
CMD="python3 bench.py --steps 6 --warmup 2 --no-ba --no-pose --no-tracking --no-cpu-baseline --no-all-cores --pipelined-streams 0 --profile 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_LDS -d gpurun_out/pmc_sq -o run --output-format csv -- $CMD > /dev/null 2> gpurun_out/pmc_sq.err
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC -d gpurun_out/pmc_sq2 -o run --output-format csv -- $CMD > /dev/null 2> gpurun_out/pmc_sq2.err
find gpurun_out/pmc_sq gpurun_out/pmc_sq2 -name '*.csv' ! -name run_counter_collection.csv -delete
