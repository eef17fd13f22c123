set -eo pipefail
export TMPDIR=/tmp
# final GPU check: the whole GPU suite
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/pytest_all.log 2>&1
