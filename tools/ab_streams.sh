# Default bench (no CPU baseline) alternating stream counts on one box.
set -e
mkdir -p gpurun_out
for s in 2 4 2 4 3; do
  timeout -k 10 300 python bench.py --no-cpu --streams $s > gpurun_out/abs.json 2>/dev/null
  python -c "
import json;d=json.loads(open('gpurun_out/abs.json').read().strip().splitlines()[-1]);print('streams=$s', d['value'], d['ms_per_step'])" >> gpurun_out/abs.txt
done
