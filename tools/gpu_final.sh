# Round-end evidence: full GPU suite, default bench (with the CPU baseline), rocprofv3 stats + PMC passes.
set -e
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err
bash tools/profile_round.sh final
