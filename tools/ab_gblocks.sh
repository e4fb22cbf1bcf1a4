# A/B of the HBM-scratch giant kernel's grid (MM2G_GIANT_GBLOCKS) on C5, 1 stream.
set -e
mkdir -p gpurun_out
for g in "${@:-128 256 512}"; do
  MM2G_GIANT_GBLOCKS=$g timeout -k 10 300 python bench.py --reads 2000 --read-len 100000 --steps 2 --warmup 1 --no-cpu --streams 1 > gpurun_out/ab_gb$g.json 2>/dev/null
  python -c "
import json;d=json.loads(open('gpurun_out/ab_gb$g.json').read().strip().splitlines()[-1]);pk=d['extra']['per_kernel']
print('gblocks=$g', round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in pk.items() if v['ms_per_step'] > 1.0})" >> gpurun_out/ab_gblocks.txt
done
