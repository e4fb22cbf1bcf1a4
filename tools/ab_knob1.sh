# 1-stream per-kernel times for each value of one knob (KNOB=name VALS="a b"), then the default-bench A/B.
set -e
mkdir -p gpurun_out
: > gpurun_out/abk1.txt
for v in $VALS; do
  timeout -k 10 300 python3 bench.py --no-cpu --no-parity --resident-steps 0 --streams 1 --shares 1 --steps 3 --warmup 1 --knob $KNOB=$v $BARGS > gpurun_out/abk1.json 2>/dev/null
  python3 -c "
import json;d=json.loads(open('gpurun_out/abk1.json').read().strip().splitlines()[-1]);pk=d['extra']['per_kernel'];print('$KNOB=$v', ' '.join(f\"{k}={v['ms_per_step']:.3f}\" for k, v in pk.items() if v['ms_per_step'] > 0.05))" >> gpurun_out/abk1.txt
done
VALS="${ABVALS:-$VALS $VALS}" bash tools/ab_knob.sh
cat gpurun_out/abk1.txt gpurun_out/abk.txt
