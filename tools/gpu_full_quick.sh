# Full GPU test suite, then the 1-stream C3 A/B lines (tools/ab_quick.sh).
set -e
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests.log 2>&1
bash tools/ab_quick.sh
