set -eo pipefail
export TMPDIR=/tmp
# scratch GPU step (development)
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tracking.py "tests/test_gpu_ba.py::test_block_cache_trim_and_reuse" "tests/test_gpu_orb.py::test_describe_partial_waves" "tests/test_gpu_match.py::test_radius_match_ties" "tests/test_gpu_bow.py::test_indexed_match_stage_boundaries" > gpurun_out/pytest.log 2>&1
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 3 --no-ba --no-pose --no-all-cores --no-rbrief31 --cpu-sample-s 2 > gpurun_out/b_trk.json 2> gpurun_out/b_trk.err
MAGE_WIN_BLUR=1 timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-ba --no-pose --no-tracking --no-cpu-baseline --no-all-cores --no-rbrief31 > gpurun_out/b_win.json 2> gpurun_out/b_win.err
