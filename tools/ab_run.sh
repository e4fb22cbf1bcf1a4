# Alternating A/B of knob sets over several configurations on one GPU box
# (>= 5 alternating pairs, spread reported by tools/show_ab.py).
#   AB="knobs_a|knobs_b" CFG="c3 c2 c5" N=5 STEPS=60 bash tools/ab_run.sh TAG
# Each line of gpurun_out/TAG/ab.txt: config, knob set, Gb/s, ms/step.
set -euo pipefail
TAG=${1:-ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
Q="--no-cpu --no-parity --resident-steps 0 --iso-batches 1"
IFS='|' read -ra SETS <<< "${AB:?AB=knobs|knobs}"
for i in $(seq 1 ${N:-5}); do
  for C in ${CFG:-c3}; do
    case "$C" in
      c3) CA="--steps ${STEPS:-60} --warmup 4" ;;
      c2) CA="--preset ecoli --reads 1000 --steps ${STEPS2:-200} --warmup 4" ;;
      c5) CA="--reads 2000 --read-len 100000 --steps ${STEPS5:-8} --warmup 1" ;;
    esac
    j=0
    for K in "${SETS[@]}"; do
      KA=""; for kv in $K; do [ "$kv" = "-" ] || KA="$KA --knob $kv"; done
      f="$OUT/${C}_${j}_$i.json"
      timeout -k 10 400 python -u bench.py $Q $CA $KA > "$f" 2> "${f%.json}.err"
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" "$f" "$C" "[$K]" | tee -a "$OUT/ab.txt"
      j=$((j + 1))
    done
  done
done
echo done > "$OUT/done"
