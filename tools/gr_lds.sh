# LDS / wait counters of the headline ORB leg (two --pmc passes, kernel trace for durations).
set -eo pipefail
export TMPDIR=/tmp
ORB="python3 bench.py --steps 10 --warmup 3 --no-ba --no-pose --no-tracking --no-cpu-baseline --pipelined-streams 0 --no-all-cores --no-rbrief31"
mkdir -p gpurun_out/lds
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/lds/p1 -o run --output-format csv -- $ORB > gpurun_out/lds/p1.json 2> gpurun_out/lds/p1.err
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_INSTS_LDS_STORE_BANDWIDTH SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/lds/p2 -o run --output-format csv -- $ORB > gpurun_out/lds/p2.json 2> gpurun_out/lds/p2.err
find gpurun_out/lds -name '*.csv' ! -name run_counter_collection.csv ! -name run_kernel_trace.csv -delete
echo done
