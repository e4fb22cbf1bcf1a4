# rocprofv3 kernel stats (default bench config), a 1-stream bench, and the sort phase profile.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-cur}
ARGS="--no-parity --resident-steps 0 --steps 5 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py $ARGS > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.err
timeout -k 10 300 python3 bench.py $ARGS --streams 1 > gpurun_out/s1_$TAG.json 2> gpurun_out/s1_$TAG.err
timeout -k 10 300 python3 bench.py --no-parity --resident-steps 0 --steps 1 --warmup 0 --streams 1 --knob sort_prof=1 > gpurun_out/sp_$TAG.json 2> gpurun_out/sp_$TAG.err
