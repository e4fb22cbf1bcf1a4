# The whole GPU suite, smoke, and the default bench line (with CPU baseline and oracle parity).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-suite}
timeout -k 10 1100 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests_$TAG.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
