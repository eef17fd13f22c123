# dev: full GPU test suite, then (optional) variant timings + the SQ counter pass
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -3 gpurun_out/t_gpu.log
if [ -n "$1" ]; then bash tools/gr_abl.sh "$1"; fi
