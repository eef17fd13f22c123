# round-4 batch c: BA parity + chol timeline after the single-wave backward; matcher gate cut-off
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_match.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_ba.log 2>&1 || { tail -40 gpurun_out/t_ba.log; exit 1; }
tail -2 gpurun_out/t_ba.log
timeout -k 10 300 python -u tools/ablate_ba.py run 0 MAGE_CHOL_ABLATE=4 > gpurun_out/abl_chol.log 2>&1 || { tail -30 gpurun_out/abl_chol.log; exit 1; }
grep variant gpurun_out/abl_chol.log
timeout -k 10 300 python -u tools/abl.py run g0,g1 > gpurun_out/abl_match.log 2>&1 || { tail -30 gpurun_out/abl_match.log; exit 1; }
tail -3 gpurun_out/abl_match.log
echo all-done
