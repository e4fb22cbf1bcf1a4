# A/B: dynamic LDS of k_sort_read (co-residency of other kernels in 2-stream mode).
set -e
mkdir -p gpurun_out
for kb in 0 136 112 96; do
  timeout -k 10 300 python3 bench.py --no-parity --resident-steps 0 --knob sort_lds_kb=$kb > gpurun_out/lds_$kb.json 2> gpurun_out/lds_$kb.err
done
timeout -k 10 300 python3 bench.py --no-parity --resident-steps 0 --streams 1 --knob sort_lds_kb=112 > gpurun_out/lds_s1_112.json 2> gpurun_out/lds_s1_112.err
