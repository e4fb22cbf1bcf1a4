# Sort phase profile (1 stream) for each experiment library name in $LIBS ("-" = the default build).
set -e
mkdir -p gpurun_out
for l in $LIBS; do
  if [ "$l" = "-" ]; then unset MM2G_LIB; else export MM2G_LIB=$PWD/minimap2_rs_amd/build/libmm2g_$l.so; fi
  timeout -k 10 300 python3 bench.py --no-cpu --no-parity --resident-steps 0 --streams 1 --shares 1 --steps 1 --warmup 1 --knob sort_prof=1 $BARGS > gpurun_out/spx.json 2> gpurun_out/spx_$l.err
  echo "$l $(grep 'sort_prof\] reads' gpurun_out/spx_$l.err | tail -1 | sed 's/.*us\/read://')"
done
