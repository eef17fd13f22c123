# dev: the default bench line (stdout JSON -> gpurun_out/bench.json)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
