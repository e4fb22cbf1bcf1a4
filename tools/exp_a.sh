set -e
mkdir -p gpurun_out/exp3
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "sketch or lazy_dp" > gpurun_out/exp3/t_sketch.log 2>&1
tail -2 gpurun_out/exp3/t_sketch.log
timeout -k 10 300 python -u bench.py --no-cpu --no-parity --resident-steps 0 --steps 1 --warmup 0 --streams 1 --shares 1 --knob sort_prof=1 > gpurun_out/exp3/sp.json 2> gpurun_out/exp3/sp.err
grep "us/read" gpurun_out/exp3/sp.err | head -1
timeout -k 10 400 python -u bench.py --no-cpu --no-parity --resident-steps 0 --steps 6 --warmup 1 --streams 1 --shares 1 > gpurun_out/exp3/s1.json 2> gpurun_out/exp3/s1.err
timeout -k 10 400 python -u bench.py --no-cpu --no-parity --resident-steps 0 --steps 16 > gpurun_out/exp3/quick.json 2> gpurun_out/exp3/quick.err
timeout -k 10 400 python -u bench.py --no-cpu --no-parity --resident-steps 0 --steps 16 --knob sketch_view=0 > gpurun_out/exp3/quick_nov.json 2> gpurun_out/exp3/quick_nov.err
