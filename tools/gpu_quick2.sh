# Kernel change check: the named GPU tests, then 1-stream per-kernel times (3 steps) twice.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${TFILES:-tests/test_gpu_parity.py tests/test_gpu_stages.py} -k "${TK:-sketch or pipeline or nt4}" > gpurun_out/q2.log 2>&1
for i in 1 2; do
timeout -k 10 300 python3 bench.py --no-cpu --no-parity --resident-steps 0 --streams 1 --shares 1 --steps 3 --warmup 1 $BARGS > gpurun_out/q2_s1_$i.json 2>/dev/null
done
python3 - <<'PY'
import json
for i in (1, 2):
    d = json.loads(open(f"gpurun_out/q2_s1_{i}.json").read().strip().splitlines()[-1])
    pk = d["extra"]["per_kernel"]
    print(" ".join(f"{k}={v['ms_per_step']:.3f}" for k, v in pk.items() if v["ms_per_step"] > 0.05))
PY
