# Chain change check: production-vs-oracle GPU tests, 1-stream per-kernel times, default bench with oracle parity.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stages.py tests/test_gpu_configs.py -k "${TK:-lazy or pipeline or dense or chunk or giant or golden or chain_batch or wide or singleton or c2 or c3 or c5}" > gpurun_out/q3.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --no-parity --resident-steps 0 --streams 1 --shares 1 --steps 3 --warmup 1 $BARGS > gpurun_out/q3_s1.json 2>/dev/null
timeout -k 10 400 python3 bench.py --no-cpu --resident-steps 0 $BARGS > gpurun_out/q3_par.json 2>/dev/null
python3 - <<'PY'
import json
for f in ("gpurun_out/q3_s1.json", "gpurun_out/q3_par.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    pk = d["extra"]["per_kernel"]
    print(f, d["value"], d["ms_per_step"], " ".join(f"{k}={v['ms_per_step']:.3f}" for k, v in pk.items() if v["ms_per_step"] > 0.04))
    p = d["extra"].get("parity_vs_oracle")
    if p: print("parity", p["identical"], p["per_read_outcome_identical"], p["reads"])
PY
