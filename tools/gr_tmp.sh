set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/pytest.log 2>&1
timeout -k 10 600 python3 bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
