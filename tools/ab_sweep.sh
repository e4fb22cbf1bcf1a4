# Several knob A/Bs in one box call: SWEEP="knob:v1 v2 v3;knob2:..." bash tools/ab_sweep.sh
set -e
mkdir -p gpurun_out
: > gpurun_out/sweep.txt
IFS=';' read -ra PARTS <<< "$SWEEP"
for part in "${PARTS[@]}"; do
  KNOB=${part%%:*}; VALS=${part#*:}
  for v in $VALS; do
    KA=""; [ "$v" != "-" ] && KA="--knob $KNOB=$v"
    timeout -k 10 300 python bench.py --no-cpu --no-parity --steps ${STEPS:-10} --resident-steps 0 $KA $BARGS > gpurun_out/sw.json 2>/dev/null
    python -c "
import json;d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]);print('$KNOB=$v', d['value'], d['ms_per_step'])" >> gpurun_out/sweep.txt
  done
done
