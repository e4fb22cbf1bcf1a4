"""Per-kernel HBM traffic from two rocprofv3 PMC passes (counters collected in
separate runs, as MI355X_MICROARCH.md §HBM / §rocprofv3 PMC slots prescribe:
FETCH_SIZE and WRITE_SIZE do not fit one pass).

    python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> \
        [--out profiles/pmc_traffic.json] [--cmd "..."]

FETCH_SIZE / WRITE_SIZE are in KiB.  gfx950 correction: FETCH_SIZE counts
half the bytes of wide coalesced reads (TCC_EA0_RDREQ x 64 B for 128-B
requests), so HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE.  Infinity-Cache hits
are counted, not excluded (same section).  bench.py reads the result as the
roofline's `traffic` for its dominant kernel (the instantiation that ran).
"""
from __future__ import annotations

import argparse
import csv
import hashlib
import json
import os
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_sha() -> str:
    """Same hash as bench.py kernel_sha(): the kernel sources the counters were taken on."""
    h = hashlib.sha256()
    for f in ("mm2g_kernels.hip", "mm2g_internal.h"):
        with open(os.path.join(ROOT, "minimap2_rs_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def per_kernel(path: str, counter: str):
    acc = defaultdict(list)
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if row["Counter_Name"] != counter:
                continue
            # template instantiations stay apart (k_sketch<true, SeqNt4, false> of the
            # query path vs k_sketch<..., SeqAscii, ...> of the index build)
            name = row["Kernel_Name"].replace("void ", "", 1).replace("(anonymous namespace)::", "").split("(")[0].strip()
            acc[name].append(float(row["Counter_Value"]) * 1024.0)
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--out", default="profiles/pmc_traffic.json")
    ap.add_argument("--cmd", default="")
    ap.add_argument("--config", default="", help='bench config the counters were taken with, e.g. "reads=10000,streams=3,scale=1.0"')
    a = ap.parse_args()
    f = per_kernel(a.fetch_csv, "FETCH_SIZE")
    w = per_kernel(a.write_csv, "WRITE_SIZE")
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate runs, --kernel-trace)",
           "correction": "hbm_bytes = 2 x FETCH_SIZE + WRITE_SIZE (gfx950: FETCH_SIZE = half of wide-read bytes)",
           "command": a.cmd, "bench_config": a.config, "kernels_sha": kernel_sha(), "kernels": {}}
    for k in sorted(set(f) | set(w)):
        fb, fn = f.get(k, (0.0, 0))
        wb, wn = w.get(k, (0.0, 0))
        out["kernels"][k] = {"fetch_bytes_per_launch": round(fb), "write_bytes_per_launch": round(wb),
                             "hbm_bytes_per_launch": round(2 * fb + wb), "launches": [fn, wn]}
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    for k, v in sorted(out["kernels"].items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"])[:12]:
        print(f"{k:40s} fetch {v['fetch_bytes_per_launch'] / 1e6:10.1f} MB  write {v['write_bytes_per_launch'] / 1e6:10.1f} MB  hbm {v['hbm_bytes_per_launch'] / 1e6:10.1f} MB")


if __name__ == "__main__":
    main()
