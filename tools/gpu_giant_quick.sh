# Giant tests, then C5 and C3 1-stream lines with the chain kernels' per-step ms.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "giant or filtered_sort or dense" > gpurun_out/giant_tests.log 2>&1
timeout -k 10 400 python bench.py --reads 2000 --read-len 100000 --steps 2 --warmup 1 --no-cpu --streams 1 > gpurun_out/gq_c5.json 2>/dev/null
timeout -k 10 300 python bench.py --no-cpu --streams 1 --steps 5 --warmup 1 > gpurun_out/gq_c3.json 2>/dev/null
for f in gq_c5 gq_c3; do
python -c "
import json;d=json.loads(open('gpurun_out/$f.json').read().strip().splitlines()[-1]);pk=d['extra']['per_kernel']
print('$f', round(d['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in pk.items() if 'long' in k or 'giant' in k})" >> gpurun_out/gq.txt
done
