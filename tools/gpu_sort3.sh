# Sort parity tests, then the 1-stream phase profile and the default bench at two LDS budgets.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stages.py -k "${TK:-filtered_sort or sort_many or dense or pipeline or singleton or seed_batch or wide_gaps}" > gpurun_out/t3.log 2>&1
for kb in 0 77; do
timeout -k 10 300 python3 bench.py --no-cpu --no-parity --resident-steps 0 --streams 1 --shares 1 --steps 3 --warmup 1 --knob sort_prof=1 --knob sort_lds_kb=$kb > gpurun_out/sp3_$kb.json 2> gpurun_out/sp3_$kb.err
done
KNOB=sort_lds_kb VALS="0 77 0 77" STEPS=12 bash tools/ab_knob.sh
