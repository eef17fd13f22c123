set -eo pipefail
export TMPDIR=/tmp
# scratch GPU step (development): full GPU suite, then the default bench line
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/pytest.log 2>&1
timeout -k 10 600 python3 -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
