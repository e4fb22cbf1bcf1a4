# A/B of one context knob over values (default bench, no CPU leg, no parity), alternating on one box.
# KNOB=name VALS="a b c" [BARGS=...] bash tools/ab_knob.sh
set -e
mkdir -p gpurun_out
: > gpurun_out/abk.txt
for v in $VALS; do
  KA=""; [ "$v" != "-" ] && KA="--knob $KNOB=$v"
  timeout -k 10 300 python bench.py --no-cpu --no-parity --steps ${STEPS:-10} $KA $BARGS > gpurun_out/abk.json 2>/dev/null
  python -c "
import json;d=json.loads(open('gpurun_out/abk.json').read().strip().splitlines()[-1]);print('$KNOB=$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], (d['extra']['resident_in_hbm'] or {}).get('ms_per_step'))" >> gpurun_out/abk.txt
done
