set -e
mkdir -p gpurun_out/exp4
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/exp4/gpu_tests.log 2>&1 || { tail -30 gpurun_out/exp4/gpu_tests.log; exit 1; }
tail -2 gpurun_out/exp4/gpu_tests.log
timeout -k 10 300 python -u bench.py --no-cpu --no-parity --resident-steps 0 --steps 1 --warmup 0 --streams 1 --shares 1 --knob sort_prof=1 > gpurun_out/exp4/sp.json 2> gpurun_out/exp4/sp.err
grep "sort_prof" gpurun_out/exp4/sp.err | tail -3
timeout -k 10 400 python -u bench.py --no-cpu --no-parity --resident-steps 0 --steps 6 --warmup 1 --streams 1 --shares 1 > gpurun_out/exp4/s1.json 2> gpurun_out/exp4/s1.err
timeout -k 10 400 python -u bench.py --no-cpu --no-parity --resident-steps 0 --steps 16 > gpurun_out/exp4/quick.json 2> gpurun_out/exp4/quick.err
timeout -k 10 400 python -u bench.py --no-cpu --no-parity --resident-steps 0 --steps 16 --knob sketch_view=0 > gpurun_out/exp4/quick_nov.json 2> gpurun_out/exp4/quick_nov.err
