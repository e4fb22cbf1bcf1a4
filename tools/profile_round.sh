#!/bin/bash
# rocprofv3 evidence for the current default bench configuration (run on the GPU box):
#   1. --kernel-trace --stats  -> per-kernel time summary
#   2. --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes -> HBM bytes per
#      launch (tools/pmc_traffic.py applies the gfx950 FETCH_SIZE correction)
# Outputs under gpurun_out/prof_<tag>/; copy the summaries to profiles/ afterwards.
set -euo pipefail
TAG=${1:-cur}
ARGS=${BENCH_ARGS:-"--no-cpu --steps 3 --warmup 1"}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py $ARGS > $OUT/stats.json 2> $OUT/stats.err
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmcF -o run -- python3 bench.py $ARGS > $OUT/pmcF.json 2> $OUT/pmcF.err
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmcW -o run -- python3 bench.py $ARGS > $OUT/pmcW.json 2> $OUT/pmcW.err
echo done
