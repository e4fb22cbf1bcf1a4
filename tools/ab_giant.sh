# A/B of the giant-segment threshold (MM2G_GIANT_MIN) on the default bench workload.
# usage: bash tools/ab_giant.sh [thresholds...]   (run on the GPU box)
set -e
mkdir -p gpurun_out
for g in "${@:-1024 1000000}"; do
  MM2G_GIANT_MIN=$g timeout -k 10 200 python bench.py --streams 1 --steps 5 --warmup 1 --no-cpu > gpurun_out/ab_g$g.json 2>/dev/null
  python -c "
import json;d=json.loads(open('gpurun_out/ab_g$g.json').read().strip().splitlines()[-1]);pk=d['extra']['per_kernel']
print('giant_min=$g', round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in pk.items() if 'chain' in k})" >> gpurun_out/ab_giant.txt
done
