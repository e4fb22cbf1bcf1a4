# Sort kernel phase profile only (MM2G_SORT_PROF), 1 stream, 1 step.
set -e
mkdir -p gpurun_out
MM2G_SORT_PROF=1 timeout -k 10 200 python bench.py --streams 1 --steps 1 --warmup 0 --no-cpu > gpurun_out/sp.json 2> gpurun_out/sp.err
