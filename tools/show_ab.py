"""Summarise tools/ab_run.sh output: per (config, knob set) the runs, mean, median and spread."""
import statistics
import sys
from collections import defaultdict

rows = defaultdict(list)
for ln in open(sys.argv[1]):
    p = ln.split()
    if len(p) < 4 or ln.startswith("#"):
        continue
    cfg, ks, v = p[0], " ".join(p[1:-2]), float(p[-2])
    rows[(cfg, ks)].append(v)
for (cfg, ks), v in sorted(rows.items()):
    print(f"{cfg:3s} {ks:40s} n={len(v)} mean={statistics.mean(v):.3f} median={statistics.median(v):.3f} "
          f"min={min(v):.3f} max={max(v):.3f} runs={' '.join(f'{x:.2f}' for x in v)}")
