# round-4 batch: BA / match / tracking parity tests, chol + matcher ablations, benches, profiles
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" || { echo "step $name failed rc=$?"; exit 1; }; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_ba.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_ba.log 2>&1 || { tail -40 gpurun_out/t_ba.log; exit 1; }
tail -2 gpurun_out/t_ba.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_tracking.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_trk.log 2>&1 || { tail -40 gpurun_out/t_trk.log; exit 1; }
tail -2 gpurun_out/t_trk.log
timeout -k 10 300 python -u tools/abl.py run g0,g1 > gpurun_out/abl_match.log 2>&1 || { tail -30 gpurun_out/abl_match.log; exit 1; }
tail -4 gpurun_out/abl_match.log
timeout -k 10 300 python -u tools/ablate_ba.py run 0 MAGE_CHOL_ABLATE=2 MAGE_CHOL_ABLATE=4 > gpurun_out/abl_chol.log 2>&1 || { tail -30 gpurun_out/abl_chol.log; exit 1; }
grep variant gpurun_out/abl_chol.log
step bench timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-all-cores --no-rbrief31 > gpurun_out/b_chol.json 2> gpurun_out/b_chol.err
step noprof timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-ba --no-pose --no-tracking --no-cpu-baseline --no-all-cores --no-rbrief31 --profile 0 --pipelined-streams 0 > gpurun_out/b_noprof.json 2> gpurun_out/b_noprof.err
step s2 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-ba --no-pose --no-tracking --no-cpu-baseline --no-all-cores --no-rbrief31 --streams 2 --pipelined-streams 0 > gpurun_out/b_s2.json 2> gpurun_out/b_s2.err
step trk timeout -k 10 200 python3 -u tools/track_kernels.py 240 > gpurun_out/track_kernels.json 2> gpurun_out/track_kernels.err
step tr31 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr31 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-ba --no-pose --no-tracking --no-cpu-baseline --pipelined-streams 0 --no-all-cores --orb-variant rbrief31 > gpurun_out/tr31.log 2>&1
find gpurun_out/tr31 -name '*.csv' ! -name run_kernel_stats.csv -delete
echo all-done
