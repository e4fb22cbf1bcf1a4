set -e
O=gpurun_out/exp6
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
Q="--no-cpu --no-parity --resident-steps 0"
timeout -k 10 300 python -u bench.py $Q --steps 1 --warmup 0 --streams 1 --shares 1 --knob sort_prof=1 > $O/sp.json 2> $O/sp.err
grep "sort_prof" $O/sp.err | tail -3
timeout -k 10 400 python -u bench.py $Q --steps 6 --warmup 1 --streams 1 --shares 1 > $O/s1.json 2> $O/s1.err
timeout -k 10 400 python -u bench.py $Q --steps 16 > $O/quick.json 2> $O/quick.err
timeout -k 10 400 python -u bench.py $Q --steps 16 --knob sketch_view=0 > $O/quick_nov.json 2> $O/quick_nov.err
timeout -k 10 400 python -u bench.py $Q --steps 16 --knob mw_min=256 > $O/quick_mw.json 2> $O/quick_mw.err
C2="--preset ecoli --reads 1000 --steps 10 --warmup 2 $Q"
timeout -k 10 400 python -u bench.py $C2 > $O/c2.json 2> $O/c2.err
timeout -k 10 400 python -u bench.py $C2 --knob sketch_view=0 > $O/c2_nov.json 2> $O/c2_nov.err
timeout -k 10 400 python -u bench.py $C2 --knob mw_min=1024 > $O/c2_mw.json 2> $O/c2_mw.err
