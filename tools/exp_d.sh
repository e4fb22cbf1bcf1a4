set -e
mkdir -p gpurun_out/exp5
C2="--preset ecoli --reads 1000 --steps 10 --warmup 2 --no-cpu --no-parity --resident-steps 0"
timeout -k 10 400 python -u bench.py $C2 > gpurun_out/exp5/c2.json 2> gpurun_out/exp5/c2.err
timeout -k 10 400 python -u bench.py $C2 --knob sketch_view=0 > gpurun_out/exp5/c2_nov.json 2> gpurun_out/exp5/c2_nov.err
timeout -k 10 400 python -u bench.py $C2 --knob mw_min=1024 > gpurun_out/exp5/c2_mw.json 2> gpurun_out/exp5/c2_mw.err
timeout -k 10 400 python -u bench.py $C2 --knob mw_min=512 > gpurun_out/exp5/c2_mw512.json 2> gpurun_out/exp5/c2_mw512.err
timeout -k 10 400 python -u bench.py --preset ecoli --reads 1000 --steps 10 --warmup 2 --no-cpu --knob mw_min=512 > gpurun_out/exp5/c2_mw512_par.json 2> gpurun_out/exp5/c2_mw512_par.err
