# Default C3 bench, 1 stream, chain kernels' per-step ms (run twice).
set -e
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu --streams 1 --steps 5 --warmup 1 > gpurun_out/abq.json 2>/dev/null
  python -c "
import json;d=json.loads(open('gpurun_out/abq.json').read().strip().splitlines()[-1]);pk=d['extra']['per_kernel']
print(round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in pk.items() if 'long' in k or 'giant' in k})" >> gpurun_out/abq.txt
done
