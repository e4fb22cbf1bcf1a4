# Seed-kernel unroll variants (tools/build_exp.sh libs): 1-stream kernel times, alternated on one box.
set -e
mkdir -p gpurun_out
: > gpurun_out/abs.txt
for lib in ${LIBS:-- sc8 sc2 sw16 -}; do
  LIBV=""; [ "$lib" != "-" ] && LIBV="minimap2_rs_amd/build/libmm2g_$lib.so"
  MM2G_LIB=$LIBV timeout -k 10 300 python bench.py --no-cpu --no-parity --resident-steps 0 --streams 1 --steps ${STEPS:-6} --warmup 1 > gpurun_out/abs.json 2>gpurun_out/abs.err
  python -c "
import json;d=json.loads(open('gpurun_out/abs.json').read().strip().splitlines()[-1]);pk=d['extra']['per_kernel'];print('$lib', d['value'], d['ms_per_step'], 'seed_count', pk['seed_count']['ms_per_step'], 'seed_write', pk['seed_write']['ms_per_step'])" >> gpurun_out/abs.txt
done
