set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "giant or filtered_sort or chunked" > gpurun_out/giant_tests.log 2>&1
MM2G_LSEG_PROF=1 timeout -k 10 200 python bench.py --streams 1 --steps 1 --warmup 0 --no-cpu > gpurun_out/giant_probe.log 2>&1
for g in 1024 1000000 1024 1000000; do
  MM2G_GIANT_MIN=$g timeout -k 10 200 python bench.py --streams 1 --steps 5 --warmup 1 --no-cpu > gpurun_out/ab_g$g.json 2>/dev/null
  python -c "
import json,sys;d=json.loads(open('gpurun_out/ab_g$g.json').read().strip().splitlines()[-1]);pk=d['extra']['per_kernel']
print('giant_min=$g', round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in pk.items() if 'long' in k or 'giant' in k})" >> gpurun_out/ab_giant.txt
done
