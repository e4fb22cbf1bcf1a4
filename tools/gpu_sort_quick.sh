# Sort parity tests, the sort phase profile, and the 1-stream C3 A/B lines.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "filtered_sort or dense or pipeline" > gpurun_out/sort_tests.log 2>&1
MM2G_SORT_PROF=1 timeout -k 10 200 python bench.py --streams 1 --steps 1 --warmup 0 --no-cpu > gpurun_out/sp.json 2> gpurun_out/sp.err
bash tools/ab_quick.sh
