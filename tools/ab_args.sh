# Alternate bench runs of whole argument sets on one box (quiet: no CPU leg, no parity):
#   ARGS="--streams 4|--streams 6" N=2 STEPS=60 bash tools/ab_args.sh TAG [extra bench args]
set -euo pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
IFS='|' read -ra SETS <<< "${ARGS:?ARGS=set|set}"
for i in $(seq 1 ${N:-2}); do
  j=0
  for A in "${SETS[@]}"; do
    timeout -k 10 300 python -u bench.py --no-cpu --no-parity --resident-steps 0 --steps ${STEPS:-60} $A "$@" > "$OUT/a_${j}_$i.json" 2> "$OUT/a_${j}_$i.err"
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" "$OUT/a_${j}_$i.json" "[$A]" | tee -a "$OUT/ab.txt"
    j=$((j + 1))
  done
done
