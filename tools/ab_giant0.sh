# Giant tests (both modes), then C5 and C3 1-stream lines with pass 0's exact-mode giant at MM2G_GIANT_MIN0 thresholds.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "giant or dense" > gpurun_out/giant_tests.log 2>&1
for g in 2048 1000000; do
  MM2G_GIANT_MIN0=$g timeout -k 10 400 python bench.py --reads 2000 --read-len 100000 --steps 2 --warmup 1 --no-cpu --streams 1 > gpurun_out/g0_c5_$g.json 2>/dev/null
  python -c "
import json;d=json.loads(open('gpurun_out/g0_c5_$g.json').read().strip().splitlines()[-1]);pk=d['extra']['per_kernel']
print('C5 min0=$g', round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in pk.items() if 'long' in k or 'giant' in k})" >> gpurun_out/g0.txt
done
for g in 256 2048; do
  MM2G_GIANT_MIN0=$g timeout -k 10 300 python bench.py --no-cpu --streams 1 --steps 5 --warmup 1 > gpurun_out/g0_c3_$g.json 2>/dev/null
  python -c "
import json;d=json.loads(open('gpurun_out/g0_c3_$g.json').read().strip().splitlines()[-1]);pk=d['extra']['per_kernel']
print('C3 min0=$g', round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in pk.items() if 'long' in k or 'giant' in k})" >> gpurun_out/g0.txt
done
