"""Time the GPU index build of the hg38-shaped reference (argv: the flags to
build, in order; default "0 0 1": non-HPC twice, the first paying one-time
initialisation, then HPC); phase times from MM2G_IKNOB_IXPROF on stderr;
prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import minimap2_rs_amd as M  # noqa: E402
from tools import simdata  # noqa: E402

flags = [int(x) for x in sys.argv[1:]] or [0, 0, 1]
names, lens, gbuf = simdata.genome("hg38", 1.0, 38, threads=16)
M.set_index_knob("ixprof", 1)
M.set_index_knob("gpu_strict", 1)
out = {"ref_bases": int(lens.sum()), "builds": []}
for flag in flags:
    t0 = time.time()
    idx = M.Index.build_from_buffer(names, gbuf, lens, w=10, k=15, b=14, flag=flag, threads=16, device=0)
    out["builds"].append({"flag": flag, "s": round(time.time() - t0, 3), "stats": list(idx.stats())})
    print(f"[ixbuild] flag {flag}: {out['builds'][-1]['s']} s", file=sys.stderr, flush=True)
    del idx
print(json.dumps(out))
