set -e
mkdir -p gpurun_out/exp3
timeout -k 10 400 python -u bench.py --preset ecoli --reads 1000 --steps 10 --warmup 2 --no-cpu > gpurun_out/exp3/c2.json 2> gpurun_out/exp3/c2.err
timeout -k 10 400 python -u bench.py --preset ecoli --reads 1000 --steps 10 --warmup 2 --no-cpu --no-parity --knob sketch_view=0 > gpurun_out/exp3/c2_nov.json 2> gpurun_out/exp3/c2_nov.err
timeout -k 10 400 python -u bench.py --reads 2000 --read-len 100000 --steps 1 --warmup 0 --streams 1 --shares 1 --no-cpu --no-parity --resident-steps 0 --knob lseg_prof=1 > gpurun_out/exp3/c5prof.json 2> gpurun_out/exp3/c5prof.err
grep -E "long_prof|lseg_prof" gpurun_out/exp3/c5prof.err | head -6
timeout -k 10 600 python -u bench.py --reads 2000 --read-len 100000 --steps 3 --warmup 1 --no-cpu --knob mw_min=4096 > gpurun_out/exp3/c5mw.json 2> gpurun_out/exp3/c5mw.err
timeout -k 10 600 python -u bench.py --reads 2000 --read-len 100000 --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/exp3/c5.json 2> gpurun_out/exp3/c5.err
