# round-end GPU pass: the whole GPU suite, then the per-row profile set and the final bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_gpu_final.log 2>&1 || { tail -30 gpurun_out/t_gpu_final.log; exit 1; }
tail -2 gpurun_out/t_gpu_final.log
bash tools/profile_round.sh ${1:-r4b} rows
echo all-done
