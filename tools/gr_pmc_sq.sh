# SQ stall counters of the ORB-only bench (dev): one --pmc pass, kernels summarised per wave
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
CMD="python3 bench.py --steps 10 --warmup 3 --no-ba --no-pose --no-tracking --no-cpu-baseline --pipelined-streams 0 --no-all-cores"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/pmc_sq -o run --output-format csv -- $CMD > gpurun_out/pmc_sq.log 2>&1
find gpurun_out/pmc_sq -name '*.csv' ! -name run_counter_collection.csv -delete
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-ba --no-pose --no-tracking --no-cpu-baseline --pipelined-streams 0 --no-all-cores > gpurun_out/b_orb.json 2> gpurun_out/b_orb.err
