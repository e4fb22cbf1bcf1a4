# Quick check after a kernel change: targeted GPU tests, then 1- and 2-stream bench lines (no CPU leg).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-q}
timeout -k 10 600 python -u -m pytest -v --maxfail=3 --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stages.py -k "${TK:-pipeline or mid_occ or remap}" > gpurun_out/tq_$TAG.log 2>&1
timeout -k 10 300 python3 bench.py --no-parity --resident-steps 0 --streams 1 $BARGS > gpurun_out/s1_$TAG.json 2> gpurun_out/s1_$TAG.err
timeout -k 10 300 python3 bench.py --no-parity --resident-steps 0 $BARGS > gpurun_out/s2_$TAG.json 2> gpurun_out/s2_$TAG.err
