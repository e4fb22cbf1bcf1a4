# A/B: keys in flight per thread in the sort passes (U=8 default lib vs U=16 build), sort phase profile + 1-stream bench.
set -e
mkdir -p gpurun_out
for v in base u16; do
  if [ $v = u16 ]; then export MM2G_LIB=$PWD/minimap2_rs_amd/build/u16/libmm2g.so; fi
  timeout -k 10 300 python3 bench.py --no-parity --resident-steps 0 --steps 1 --warmup 0 --streams 1 --knob sort_prof=1 > gpurun_out/sp_$v.json 2> gpurun_out/sp_$v.err
  timeout -k 10 300 python3 bench.py --no-parity --resident-steps 0 --streams 1 > gpurun_out/s1_$v.json 2> gpurun_out/s1_$v.err
done
