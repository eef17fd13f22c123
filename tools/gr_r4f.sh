# round-4 batch f: column-fixed band resize — ORB / image parity, then the ORB profiling sets
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_image.py tests/test_stereo_scale.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_orb.log 2>&1 || { tail -40 gpurun_out/t_orb.log; exit 1; }
tail -2 gpurun_out/t_orb.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-ba --no-pose --no-tracking --no-cpu-baseline --no-all-cores --pipelined-streams 0 > gpurun_out/b_orb.json 2> gpurun_out/b_orb.err || { tail -20 gpurun_out/b_orb.err; exit 1; }
bash tools/profile_round.sh r4 main || exit 1
echo all-done
