# Contexts x units per batch x HIP hardware queues per process x kernel library,
# default bench (no CPU baseline, no parity), alternated on one box.
# Each cfg is "streams shares hwq lib" (lib: "-" = libmm2g.so, else libmm2g_<lib>.so).
set -e
mkdir -p gpurun_out
: > gpurun_out/abq.txt
IFS=, ; for cfg in ${CFGS:-4 2 4 -,6 3 8 -,8 4 8 -,4 2 8 -,4 2 4 wpe6,4 2 4 -}; do IFS=" "
  set -- $cfg
  LIBV=""; [ "$4" != "-" ] && LIBV="minimap2_rs_amd/build/libmm2g_$4.so"
  MM2G_LIB=$LIBV GPU_MAX_HW_QUEUES=$3 timeout -k 10 300 python bench.py --no-cpu --no-parity --resident-steps 0 --steps ${STEPS:-16} --streams $1 --shares $2 > gpurun_out/abq.json 2>gpurun_out/abq.err
  python -c "
import json;d=json.loads(open('gpurun_out/abq.json').read().strip().splitlines()[-1]);pk=d['extra']['per_kernel'];print('streams=$1 shares=$2 hwq=$3 lib=$4', d['value'], d['ms_per_step'], d['extra']['host_ms_per_unit'], 'sketch', pk['sketch']['ms_per_step'])" >> gpurun_out/abq.txt
done
