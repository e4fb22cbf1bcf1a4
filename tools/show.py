"""Print bench lines (value, ms/step, host timings, per-kernel ms) from gpurun_out/*.json."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.load(open(f))
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable", e)
        continue
    x = d["extra"]
    print(f"{f}: {d['value']:.3f} Gb/s  {d['ms_per_step']:.2f} ms/step  host {x.get('host_ms_per_unit')}  roof {d['roofline']['kernel']} {d['roofline']['frac']:.3f}")
    pk = x["per_kernel"]
    print("   ", {k: round(v["ms_per_step"], 3) for k, v in sorted(pk.items(), key=lambda kv: -kv[1]["ms_per_step"])})
