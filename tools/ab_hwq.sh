# Contexts x units per batch x HIP hardware queues per process, default bench (no CPU
# baseline, no parity), alternated on one box.  Each cfg is "streams shares hwq".
set -e
mkdir -p gpurun_out
: > gpurun_out/abq.txt
IFS=, ; for cfg in ${CFGS:-4 2 4,6 3 8,8 4 8,4 2 8,4 2 4}; do IFS=" "
  set -- $cfg
  GPU_MAX_HW_QUEUES=$3 timeout -k 10 300 python bench.py --no-cpu --no-parity --resident-steps 0 --steps ${STEPS:-16} --streams $1 --shares $2 > gpurun_out/abq.json 2>gpurun_out/abq.err
  python -c "
import json;d=json.loads(open('gpurun_out/abq.json').read().strip().splitlines()[-1]);print('streams=$1 shares=$2 hwq=$3', d['value'], d['ms_per_step'], d['extra']['host_ms_per_unit'])" >> gpurun_out/abq.txt
done
