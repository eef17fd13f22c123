set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py "tests/test_gpu_ba.py::test_repeated_setters_before_a_step" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_match.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-ba --no-pose --no-tracking --no-cpu-baseline --pipelined-streams 0 --no-all-cores > gpurun_out/b_orb.json 2> gpurun_out/b_orb.err
