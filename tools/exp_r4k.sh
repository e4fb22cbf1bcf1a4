set -e
O=gpurun_out/r4k; mkdir -p $O
C2="--preset ecoli --reads 1000 --steps 10 --warmup 2 --no-cpu --no-parity --resident-steps 0 --streams 1 --shares 1"
for i in 1 2; do
for K in 0 256 1024; do
  timeout -k 10 300 python -u bench.py $C2 --knob mw_min=$K > $O/c2s1_mw${K}_$i.json 2> $O/c2s1_mw${K}_$i.err
  python3 - $O/c2s1_mw${K}_$i.json $K <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk = d["extra"]["per_kernel"]
print("mw_min", sys.argv[2], d["value"], d["ms_per_step"], {k: round(v["ms_per_step"], 3) for k, v in pk.items() if "long" in k or "sketch" in k})
PY
done
done
