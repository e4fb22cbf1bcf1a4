# Contexts (streams) vs units per batch, default bench (no CPU baseline, no parity), on one box.
set -e
mkdir -p gpurun_out
: > gpurun_out/abc.txt
IFS=, ; for cfg in ${CFGS:-2 2,3 2,4 2}; do IFS=" "
  set -- $cfg
  timeout -k 10 300 python bench.py --no-cpu --no-parity --steps ${STEPS:-10} --streams $1 --shares $2 > gpurun_out/abc.json 2>/dev/null
  python -c "
import json;d=json.loads(open('gpurun_out/abc.json').read().strip().splitlines()[-1]);print('streams=$1 shares=$2', d['value'], d['ms_per_step'], d['extra']['host_ms_per_unit'], (d['extra']['resident_in_hbm'] or {}).get('ms_per_step'))" >> gpurun_out/abc.txt
done
