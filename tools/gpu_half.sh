# k_chain_long2 check: parity + stage suites, then 1-stream A/B (chain_half 0/1) and a 2-stream line.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --maxfail=3 --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stages.py > gpurun_out/th.log 2>&1
for h in 0 1; do
  timeout -k 10 300 python3 bench.py --no-parity --resident-steps 0 --streams 1 --knob chain_half=$h > gpurun_out/s1_h$h.json 2> gpurun_out/s1_h$h.err
done
timeout -k 10 300 python3 bench.py --no-parity --resident-steps 0 > gpurun_out/s2_h1.json 2> gpurun_out/s2_h1.err
