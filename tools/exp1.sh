set -e
mkdir -p gpurun_out/exp2
for m in 3 1; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-parity --resident-steps 0 --steps 1 --warmup 0 --streams 1 --shares 1 --knob sort_prof=1 --knob sort_lb=$m > gpurun_out/exp2/sp$m.json 2> gpurun_out/exp2/sp$m.err
  grep "us/read" gpurun_out/exp2/sp$m.err | head -1
done
timeout -k 10 400 python -u bench.py --no-cpu --no-parity --resident-steps 0 --steps 6 --warmup 1 --streams 1 --shares 1 > gpurun_out/exp2/s1.json 2> gpurun_out/exp2/s1.err
timeout -k 10 400 python -u bench.py --no-cpu --no-parity --resident-steps 0 --steps 16 > gpurun_out/exp2/quick.json 2> gpurun_out/exp2/quick.err
