# Round evidence: the whole GPU suite, smoke, the default bench line, rocprofv3 kernel stats of the default bench.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-full}
timeout -k 10 1100 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests_$TAG.log 2>&1 || echo "GPU TESTS FAILED rc=$?" >> gpurun_out/gpu_tests_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --no-parity --resident-steps 0 > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.err
