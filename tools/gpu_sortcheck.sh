# Sort change check: sort parity tests, sort phase profile, 1- and 2-stream bench.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-x}
timeout -k 10 600 python -u -m pytest -v --maxfail=3 --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "sort or singleton or pipeline" > gpurun_out/ts_$TAG.log 2>&1
timeout -k 10 300 python3 bench.py --no-parity --resident-steps 0 --steps 1 --warmup 0 --streams 1 --knob sort_prof=1 > gpurun_out/sp_$TAG.json 2> gpurun_out/sp_$TAG.err
timeout -k 10 300 python3 bench.py --no-parity --resident-steps 0 --streams 1 > gpurun_out/s1_$TAG.json 2> gpurun_out/s1_$TAG.err
timeout -k 10 300 python3 bench.py --no-parity --resident-steps 0 > gpurun_out/s2_$TAG.json 2> gpurun_out/s2_$TAG.err
