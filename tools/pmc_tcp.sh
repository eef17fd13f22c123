set -eo pipefail
export TMPDIR=/tmp
CMD="python3 bench.py --steps 6 --warmup 2 --no-ba --no-pose --no-tracking --no-cpu-baseline --no-all-cores --pipelined-streams 0 --profile 0"
timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TA_BUSY_avr -d gpurun_out/pmc_tcp -o run --output-format csv -- $CMD > /dev/null 2> gpurun_out/pmc_tcp.err
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE -d gpurun_out/pmc_tcp2 -o run --output-format csv -- $CMD > /dev/null 2> gpurun_out/pmc_tcp2.err
find gpurun_out/pmc_tcp gpurun_out/pmc_tcp2 -name '*.csv' ! -name run_counter_collection.csv -delete
