# GPU-box runs of this repository, one parameterized script (replaces the round-1/2
# one-off launchers).  Run through gpurun from the repo root:
#   bash tools/gpu_run.sh <step>[,<step>...] [TAG]
# Steps (each under its own time limit; the first failure ends the run):
#   suite   pytest -m gpu (whole suite) + smoke()
#   tests:<expr>  pytest -m gpu -k <expr>
#   bench   the default bench line (C3, CPU baseline + oracle parity)
#   quick   the default bench line without the CPU leg and parity (BARGS adds flags)
#   c2, c5  the C2 / C5 bench lines (oracle parity, no CPU leg)
#   multi   multi-GPU launch checks on one GPU: `--gpus 2` must fail loudly; a
#           2-rank gloo rehearsal (both ranks on the one GPU) must report ranks 2, n_gpus 1
#   s1      1-stream line (kernel times on a quiet GPU) + the sort phase profile
#   prof    rocprofv3 --kernel-trace --stats of a short default bench
#   prof1   the same with one context (--streams 1): every launch alone on the GPU, the
#           conditions of the bench line's quiet-GPU roofline figure
#   c5s1    C5 with one context and one unit per batch, with the long-segment profile
#   c3p     C3 phase profiles (one context, one unit): sketch, sort, long segments
#   pmc     FETCH_SIZE and WRITE_SIZE passes (separate runs) -> pmc_traffic.json
#   sq      one SQ counter pass (stall shares, LDS bank conflicts), 1 stream
#   ab      alternate bench runs of knob sets: AB="sort_lds_kb=157|sort_lds_kb=128" N=3
#   abdir   alternate quick bench runs of whole trees (same box): DIRS=". .ab/r02" N=2
#   ixb     GPU index build of the hg38-shaped reference, phase times (IXFLAGS="0 0 1")
# Outputs: gpurun_out/<TAG>/ (TAG defaults to "run").
set -euo pipefail
STEPS_ARG=${1:?steps}
TAG=${2:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BARGS=${BARGS:-}
QUIET="--no-cpu --no-parity --resident-steps 0"

line() {   # print the bench line's headline fields
  python3 - "$1" <<'EOF'
import json, sys
t = open(sys.argv[1]).read().strip().splitlines()
d = json.loads(t[-1]) if t else {}
r = d.get("roofline", {})
print(sys.argv[1], d.get("value"), d.get("ms_per_step"), r.get("kernel"), r.get("frac"),
      (d.get("extra", {}).get("parity_vs_oracle") or {}).get("identical"))
EOF
}

IFS=',' read -ra STEPS <<< "$STEPS_ARG"
for S in "${STEPS[@]}"; do
  case "$S" in
    suite)
      timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > "$OUT/gpu_tests.log" 2>&1
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    tests:*)
      timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ -k "${S#tests:}" > "$OUT/gpu_tests_k.log" 2>&1 ;;
    bench)
      timeout -k 10 600 python -u bench.py $BARGS > "$OUT/bench.json" 2> "$OUT/bench.err"; line "$OUT/bench.json" ;;
    quick)
      timeout -k 10 400 python -u bench.py $QUIET --steps ${N:-16} $BARGS > "$OUT/quick.json" 2> "$OUT/quick.err"; line "$OUT/quick.json" ;;
    c2)
      timeout -k 10 400 python -u bench.py --preset ecoli --reads 1000 --steps 200 --warmup 2 --no-cpu $BARGS > "$OUT/c2.json" 2> "$OUT/c2.err"; line "$OUT/c2.json" ;;
    c5)
      timeout -k 10 600 python -u bench.py --reads 2000 --read-len 100000 --steps 12 --warmup 1 --no-cpu $BARGS > "$OUT/c5.json" 2> "$OUT/c5.err"; line "$OUT/c5.json" ;;
    multi)
      rc=0; timeout -k 10 120 python -u bench.py --gpus 2 --steps 2 > "$OUT/multi_nccl2.json" 2> "$OUT/multi_nccl2.err" || rc=$?
      echo "bench.py --gpus 2 on $(python3 -c 'import torch; print(torch.cuda.device_count())') GPU(s): exit $rc" | tee "$OUT/multi_nccl2.rc"
      [ "$rc" -ne 0 ] || { echo "expected a loud failure"; exit 1; }
      MM2G_DIST_BACKEND=gloo timeout -k 10 900 python -u bench.py --gpus 2 --steps 4 --warmup 1 --streams 2 --no-cpu \
        > "$OUT/multi_gloo2.json" 2> "$OUT/multi_gloo2.err"; line "$OUT/multi_gloo2.json" ;;
    s1)
      timeout -k 10 400 python -u bench.py $QUIET --steps 6 --warmup 1 --streams 1 --shares 1 $BARGS > "$OUT/s1.json" 2> "$OUT/s1.err"; line "$OUT/s1.json"
      timeout -k 10 300 python -u bench.py $QUIET --steps 1 --warmup 0 --streams 1 --shares 1 --knob sort_prof=1 $BARGS > "$OUT/sortprof.json" 2> "$OUT/sortprof.err"
      grep sort_prof "$OUT/sortprof.err" || true ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 bench.py $QUIET --steps 6 --warmup 1 $BARGS \
        > "$OUT/prof.json" 2> "$OUT/prof.err"; line "$OUT/prof.json" ;;
    prof1)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats1" -o run -- python3 bench.py $QUIET --steps 6 --warmup 1 --streams 1 $BARGS \
        > "$OUT/prof1.json" 2> "$OUT/prof1.err"; line "$OUT/prof1.json" ;;
    c5s1)
      timeout -k 10 600 python -u bench.py $QUIET --reads 2000 --read-len 100000 --steps 3 --warmup 1 --streams 1 --shares 1 --knob lseg_prof=1 $BARGS \
        > "$OUT/c5s1.json" 2> "$OUT/c5s1.err"; line "$OUT/c5s1.json"; grep -E "_prof\]" "$OUT/c5s1.err" | cut -c1-600 > "$OUT/c5s1_prof.txt" || true ;;
    c3p)
      timeout -k 10 300 python -u bench.py $QUIET --steps 1 --warmup 1 --streams 1 --shares 1 --knob lseg_prof=1 --knob sketch_prof=1 --knob sort_prof=1 $BARGS \
        > "$OUT/c3p.json" 2> "$OUT/c3p.err"; grep -E "_prof\]" "$OUT/c3p.err" | cut -c1-900 > "$OUT/c3p_prof.txt" || true ;;
    pmc)
      timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmcF" -o run -- python3 bench.py $QUIET --steps 6 --warmup 1 $BARGS > "$OUT/pmcF.json" 2> "$OUT/pmcF.err"
      timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmcW" -o run -- python3 bench.py $QUIET --steps 6 --warmup 1 $BARGS > "$OUT/pmcW.json" 2> "$OUT/pmcW.err"
      CFG=$(python3 -c "import bench, sys; print(bench.bench_config_tag(bench.parse(sys.argv[1:])))" $BARGS)
      python3 tools/pmc_traffic.py "$OUT/pmcF/run_counter_collection.csv" "$OUT/pmcW/run_counter_collection.csv" --out "$OUT/pmc_traffic.json" \
        --config "$CFG" --cmd "rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE --kernel-trace -- python3 bench.py $QUIET --steps 6 --warmup 1 $BARGS" > "$OUT/pmc_traffic.txt" ;;
    sq)
      timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU \
        --kernel-trace --output-format csv -d "$OUT/pmcSQ" -o run -- python3 bench.py $QUIET --streams 1 --shares 1 --steps 2 --warmup 1 $BARGS > "$OUT/sq.json" 2> "$OUT/sq.err"
      python3 tools/pmc_sq.py "$OUT/pmcSQ/run_counter_collection.csv" > "$OUT/sq_summary.json" ;;
    ab)
      IFS='|' read -ra SETS <<< "${AB:?AB=knobs|knobs}"
      for i in $(seq 1 ${N:-3}); do
        j=0
        for K in "${SETS[@]}"; do
          KA=""; for kv in $K; do [ "$kv" = "-" ] || KA="$KA --knob $kv"; done
          timeout -k 10 300 python -u bench.py $QUIET --steps ${ABSTEPS:-12} $KA $BARGS > "$OUT/ab_${j}_$i.json" 2> "$OUT/ab_${j}_$i.err"
          echo "[$K] $(line "$OUT/ab_${j}_$i.json")" | tee -a "$OUT/ab.txt"
          j=$((j + 1))
        done
      done ;;
    abdir)
      for i in $(seq 1 ${N:-2}); do
        for D in ${DIRS:?DIRS=". .ab/r02"}; do
          nm=$(echo "$D" | tr -c 'a-zA-Z0-9\n' '_')
          (cd "$D" && timeout -k 10 300 python -u bench.py $QUIET --steps ${ABSTEPS:-16} $BARGS) > "$OUT/abd_${nm}_$i.json" 2> "$OUT/abd_${nm}_$i.err"
          echo "[$D] $(line "$OUT/abd_${nm}_$i.json")" | tee -a "$OUT/abdir.txt"
        done
      done ;;
    ixb)
      timeout -k 10 300 python -u tools/ixbuild_hpc_time.py ${IXFLAGS:-0 0 1} > "$OUT/ixb.json" 2> "$OUT/ixb.err"; cat "$OUT/ixb.json"; grep ixbuild "$OUT/ixb.err" || true ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
  echo "step $S done" >> "$OUT/progress.txt"
done
echo done > "$OUT/done"
