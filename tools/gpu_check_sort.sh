# After a sort/chain kernel change: sort and chain parity tests vs the oracle,
# the sort phase profile (1 stream), then two default bench lines (no CPU leg).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stages.py -k "${TK:-sort or pipeline or lazy or giant or dense or golden or chunk}" > gpurun_out/tcs.log 2>&1
LIBS="-" STEPS=4 bash tools/ab_sortu.sh
for t in 1 2; do timeout -k 10 300 python bench.py --no-cpu --no-parity --resident-steps 0 --steps 16 > gpurun_out/bcs$t.json 2> gpurun_out/bcs$t.err; done
