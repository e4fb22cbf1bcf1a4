"""hg38-scale .mmi round trip and mid_occ timings.

Builds the bench's hg38-shaped index on the GPU, writes it as .mmi, loads it
back with 1 thread and with the default thread count (mapped, bucket-parallel
loader), uploads it and computes mid_occ both ways: the host's sort of all
counts (the reference's calc_mid_occ) and the device histogram.  Prints one
JSON line.  Run on the GPU box: python tools/mmi_load_bench.py [--scale S]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import minimap2_rs_amd as M  # noqa: E402
from tools import simdata  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--path", default="/tmp/mm2g_hg38.mmi")
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    names, lens, gbuf = simdata.genome("hg38", a.scale, 38, threads=a.threads)
    t = time.time()
    idx = M.Index.build_from_buffer(names, gbuf, lens, w=10, k=15, b=14, flag=0, threads=a.threads, device=0)
    r = {"ref_gb": round(float(lens.sum()) / 1e9, 3), "build_gpu_s": round(time.time() - t, 2)}
    t = time.time()
    idx.save_to_mmi(a.path)
    r["save_s"] = round(time.time() - t, 2)
    r["file_gb"] = round(os.path.getsize(a.path) / 1e9, 3)
    st = idx.stats()
    idx.close()
    try:
        for thr in ("1", str(a.threads)):
            M.set_index_knob("load_threads", int(thr))
            t = time.time()
            back = M.Index.load_from_mmi(a.path)
            r[f"load_s_{thr}t"] = round(time.time() - t, 2)
            assert tuple(back.stats()) == tuple(st)
            if thr == "1":
                back.close()
    finally:
        os.remove(a.path)
    t = time.time()
    mh = back.calc_mid_occ(2e-4)
    r["mid_occ_host_sort_s"] = round(time.time() - t, 3)
    d = M.Device(0)
    t = time.time()
    d.upload_index(back, 10)
    r["upload_s"] = round(time.time() - t, 2)
    t = time.time()
    md = d.index_mid_occ(2e-4)
    r["mid_occ_device_s"] = round(time.time() - t, 4)
    assert md == mh, (md, mh)
    r["mid_occ"] = md
    r["n_keys"] = st[0]
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
