# One SQ counter pass (8 SQ slots) over a short 1-stream bench: where the waves' cycles go
# (WAIT_ANY = parked on s_waitcnt/barrier, WAIT_INST_ANY = issue stalls, ACTIVE_INST_ANY),
# summarized per kernel by tools/pmc_sq.py into gpurun_out/pmcSQ/summary.json.
set -e
mkdir -p gpurun_out/pmcSQ
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU \
  --kernel-trace --output-format csv -d gpurun_out/pmcSQ -o run -- python3 bench.py --no-cpu --no-parity --resident-steps 0 --streams 1 --shares 1 --steps 2 --warmup 1 > gpurun_out/pmcSQ/b.json 2> gpurun_out/pmcSQ/b.err
python3 tools/pmc_sq.py gpurun_out/pmcSQ/run_counter_collection.csv > gpurun_out/pmcSQ/summary.json
