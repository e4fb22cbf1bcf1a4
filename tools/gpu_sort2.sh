# Sort change check: sort/pipeline parity tests, the 1-stream sort phase profile, the default bench with oracle parity.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-s2}
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stages.py -k "${TK:-filtered_sort or sort_many or dense or pipeline or singleton or seed_batch or wide_gaps}" > gpurun_out/t_$TAG.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --no-parity --resident-steps 0 --streams 1 --shares 1 --steps 3 --warmup 1 --knob sort_prof=1 > gpurun_out/sp_$TAG.json 2> gpurun_out/sp_$TAG.err
timeout -k 10 400 python3 bench.py --no-cpu --resident-steps 0 $BARGS > gpurun_out/b_$TAG.json 2> gpurun_out/b_$TAG.err
