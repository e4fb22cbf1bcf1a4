# GPU tests, then the sort kernel's phase profile (MM2G_SORT_PROF) and a default bench.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests.log 2>&1
MM2G_SORT_PROF=1 timeout -k 10 200 python bench.py --streams 1 --steps 1 --warmup 0 --no-cpu > gpurun_out/sp.json 2> gpurun_out/sp.err
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err
