# C4 per-kernel times and the pose / tracking bench legs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/track_kernels.py 240 > gpurun_out/track_kernels.json 2> gpurun_out/track_kernels.err || { tail -20 gpurun_out/track_kernels.err; exit 1; }
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-ba --no-cpu-baseline --no-all-cores --no-rbrief31 --pipelined-streams 0 > gpurun_out/b_trk.json 2> gpurun_out/b_trk.err || { tail -20 gpurun_out/b_trk.err; exit 1; }
echo all-done
