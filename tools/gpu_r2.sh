# GPU parity suites (stages + parity), then a default bench line.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --maxfail=8 --timeout 300 --timeout-method thread -m gpu tests/test_gpu_stages.py tests/test_gpu_parity.py -k "${T1_K:-}" > gpurun_out/t1.log 2>&1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err
