# The whole GPU suite, then three default bench lines (no CPU leg, no parity).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/suite.log 2>&1
for t in 1 2 3; do timeout -k 10 300 python bench.py --no-cpu --no-parity --resident-steps 0 --steps 16 > gpurun_out/bsb$t.json 2> gpurun_out/bsb$t.err; done
