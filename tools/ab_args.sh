# Alternating A/B of bench.py argument sets on one GPU box (as tools/ab_run.sh, but the
# variants are bench arguments, e.g. contexts or units per batch):
#   AB="--shares 2|--shares 4" N=3 STEPS=60 bash tools/ab_args.sh TAG
# Each line of gpurun_out/TAG/ab.txt: variant, Gb/s, ms/step.
set -euo pipefail
TAG=${1:-abargs}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
Q="--no-cpu --no-parity --resident-steps 0 --iso-batches 1"
IFS='|' read -ra SETS <<< "${AB:?AB=args|args}"
for i in $(seq 1 ${N:-3}); do
  j=0
  for A in "${SETS[@]}"; do
    f="$OUT/v${j}_$i.json"
    timeout -k 10 400 python -u bench.py $Q --steps ${STEPS:-60} --warmup 4 $A > "$f" 2> "${f%.json}.err"
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c3', sys.argv[2], d['value'], d['ms_per_step'])" "$f" "[$A]" | tee -a "$OUT/ab.txt"
    j=$((j + 1))
  done
done
echo done > "$OUT/done"
