# Sort phase profile, then the default bench at 2, 3 and 4 streams (no CPU baseline).
set -e
mkdir -p gpurun_out
MM2G_SORT_PROF=1 timeout -k 10 200 python bench.py --streams 1 --steps 1 --warmup 0 --no-cpu > gpurun_out/sp.json 2> gpurun_out/sp.err
for s in 2 3 4; do
  timeout -k 10 200 python bench.py --no-cpu --streams $s > gpurun_out/bs$s.json 2> gpurun_out/bs$s.err
done
