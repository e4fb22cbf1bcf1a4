# k_sort_read pass widths (SORT_U1 / SORT_U2 builds from tools/build_exp.sh): phase
# profile (1 stream) and the sort kernel time, alternated on one box.
set -e
mkdir -p gpurun_out
: > gpurun_out/absu.txt
for lib in ${LIBS:-- u1x16 u1x24 u12x16 -}; do
  LIBV=""; [ "$lib" != "-" ] && LIBV="minimap2_rs_amd/build/libmm2g_$lib.so"
  MM2G_LIB=$LIBV timeout -k 10 300 python bench.py --no-cpu --no-parity --resident-steps 0 --streams 1 --steps ${STEPS:-4} --warmup 1 --knob sort_prof=1 > gpurun_out/absu.json 2>gpurun_out/absu.err
  echo "== $lib" >> gpurun_out/absu.txt
  grep "sort_prof\] reads" gpurun_out/absu.err | tail -2 >> gpurun_out/absu.txt
  python -c "
import json;d=json.loads(open('gpurun_out/absu.json').read().strip().splitlines()[-1]);pk=d['extra']['per_kernel'];print('$lib', d['value'], d['ms_per_step'], 'sort_large', pk['sort_large']['ms_per_step'])" >> gpurun_out/absu.txt
done
