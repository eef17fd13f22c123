set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err
