# Sort change check: sort-related GPU tests, 1-stream per-kernel times, the sort phase profile.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stages.py tests/test_gpu_configs.py -k "${TK:-pipeline or sort or singleton or chunked or c3 or c5 or seed_batch}" > gpurun_out/sq.log 2>&1
tail -1 gpurun_out/sq.log
timeout -k 10 300 python3 bench.py --no-cpu --no-parity --resident-steps 0 --streams 1 --shares 1 --steps 3 --warmup 1 $BARGS > gpurun_out/sq_s1.json 2>/dev/null
timeout -k 10 300 python3 bench.py --no-cpu --no-parity --resident-steps 0 --streams 1 --shares 1 --steps 1 --warmup 1 --knob sort_prof=1 $BARGS > gpurun_out/sq_sp.json 2> gpurun_out/sq_sp.err
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/sq_s1.json").read().strip().splitlines()[-1])
print(" ".join(f"{k}={v['ms_per_step']:.3f}" for k, v in d["extra"]["per_kernel"].items() if v["ms_per_step"] > 0.05))
PY
grep "sort_prof\] reads\|sort_prof\] keys" gpurun_out/sq_sp.err | tail -2
