# VALU issue-busy calibration: SQ_ACTIVE_INST_VALU(2) on the VALU probe (known instruction classes)
# and on the headline ORB leg, one --pmc pass each (kernel trace for durations).
set -eo pipefail
export TMPDIR=/tmp
C="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
mkdir -p gpurun_out/vbusy
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/vbusy/probe -o run --output-format csv -- ./tools/valu_probe > gpurun_out/vbusy/probe.txt 2> gpurun_out/vbusy/probe.err
timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/vbusy/orb -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-ba --no-pose --no-tracking --no-cpu-baseline --pipelined-streams 0 --no-all-cores --no-rbrief31 > gpurun_out/vbusy/orb.json 2> gpurun_out/vbusy/orb.err
find gpurun_out/vbusy -name '*.csv' ! -name run_counter_collection.csv ! -name run_kernel_trace.csv -delete
echo done
