# Giant-segment tests (LDS and HBM-scratch variants), then C5 and C3 bench lines.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "giant or filtered_sort" > gpurun_out/giant_tests.log 2>&1
timeout -k 10 500 python bench.py --reads 2000 --read-len 100000 --steps 3 --warmup 1 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err
