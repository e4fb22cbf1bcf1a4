# Round evidence on the current code (run on the GPU box; outputs under gpurun_out/ev_<tag>/):
#   the whole GPU suite, smoke, rocprofv3 --kernel-trace --stats of the default bench,
#   two separate PMC passes (FETCH_SIZE, WRITE_SIZE) -> pmc_traffic.json, then the
#   default bench line (CPU baseline + oracle parity) reading that traffic.
set -euo pipefail
TAG=${1:-cur}
OUT=gpurun_out/ev_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BARGS="--no-cpu --no-parity --resident-steps 0 --steps 6 --warmup 1"
timeout -k 10 1000 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py $BARGS > $OUT/stats.json 2> $OUT/stats.err
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmcF -o run -- python3 bench.py $BARGS > $OUT/pmcF.json 2> $OUT/pmcF.err
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmcW -o run -- python3 bench.py $BARGS > $OUT/pmcW.json 2> $OUT/pmcW.err
CFG=$(python3 -c "import bench; print(bench.bench_config_tag(bench.parse([])))")
python3 tools/pmc_traffic.py $OUT/pmcF/run_counter_collection.csv $OUT/pmcW/run_counter_collection.csv --out $OUT/pmc_traffic.json \
  --config "$CFG" --cmd "rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE --kernel-trace -- python3 bench.py $BARGS" > $OUT/pmc_traffic.txt
cp $OUT/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
echo done > $OUT/done
