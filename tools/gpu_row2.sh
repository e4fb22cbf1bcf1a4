# GPU tests for the .mmi loader / device mid_occ, then the hg38-scale round trip.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 600 python -u tools/mmi_load_bench.py > gpurun_out/mmi_load.json 2> gpurun_out/mmi_load.err
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
