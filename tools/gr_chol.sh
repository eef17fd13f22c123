# round-4 batch: BA / match / tracking parity tests, chol + matcher ablations, one bench (no CPU legs)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_ba.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_ba.log 2>&1 || { tail -40 gpurun_out/t_ba.log; exit 1; }
tail -2 gpurun_out/t_ba.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_tracking.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_trk.log 2>&1 || { tail -40 gpurun_out/t_trk.log; exit 1; }
tail -2 gpurun_out/t_trk.log
timeout -k 10 300 python -u tools/abl.py run g0,g1 > gpurun_out/abl_match.log 2>&1 || { tail -30 gpurun_out/abl_match.log; exit 1; }
tail -4 gpurun_out/abl_match.log
timeout -k 10 300 python -u tools/ablate_ba.py run 0 MAGE_CHOL_ABLATE=2 MAGE_CHOL_ABLATE=4 > gpurun_out/abl_chol.log 2>&1 || { tail -30 gpurun_out/abl_chol.log; exit 1; }
grep variant gpurun_out/abl_chol.log
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-all-cores --no-rbrief31 > gpurun_out/b_chol.json 2> gpurun_out/b_chol.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-ba --no-pose --no-tracking --no-cpu-baseline --no-all-cores --no-rbrief31 --profile 0 > gpurun_out/b_noprof.json 2> gpurun_out/b_noprof.err
