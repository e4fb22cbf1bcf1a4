"""Attribute GPU wall time to kernels from a rocprofv3 kernel trace.

With several streams, kernels overlap, so a kernel's own duration says little
about what it costs the step.  This splits every instant of the window among
the kernels running then (equal shares) and reports, per kernel name, the
attributed milliseconds, the plain summed duration, and the busy fraction of
the window.  Usage: python tools/timeline.py <kernel_trace.csv> [first_kernel_substring]
(the window starts at the first launch whose name contains the substring,
default the first nt4 sketch, i.e. after the index build).
"""
import csv
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    for p in ("void ", "(anonymous namespace)::"):
        n = n.replace(p, "")
    if "rocprim" in n:
        return "rocprim"
    return n


def main():
    path = sys.argv[1]
    start_key = sys.argv[2] if len(sys.argv) > 2 else "SeqNt4"
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    t0 = next(s for s, e, n in rows if start_key in n)
    rows = [(s, e, short(n)) for s, e, n in rows if s >= t0]
    t1 = max(e for s, e, n in rows)
    ev = []
    for k, (s, e, n) in enumerate(rows):
        ev.append((s, 1, k))
        ev.append((e, -1, k))
    ev.sort()
    live = set()
    att = defaultdict(float)
    dur = defaultdict(float)
    cnt = defaultdict(int)
    busy = 0.0
    prev = t0
    for t, d, k in ev:
        if live and t > prev:
            share = (t - prev) / len(live)
            for j in live:
                att[rows[j][2]] += share
            busy += t - prev
        prev = t
        if d > 0:
            live.add(k)
        else:
            live.discard(k)
    for s, e, n in rows:
        dur[n] += e - s
        cnt[n] += 1
    win = t1 - t0
    print(f"window {win / 1e6:.2f} ms, GPU busy {busy / win:.3f}")
    print(f"{'kernel':32s} {'attrib_ms':>10s} {'frac':>6s} {'sum_dur_ms':>10s} {'calls':>6s}")
    for n, a in sorted(att.items(), key=lambda x: -x[1]):
        print(f"{n:32s} {a / 1e6:10.2f} {a / win:6.3f} {dur[n] / 1e6:10.2f} {cnt[n]:6d}")


if __name__ == "__main__":
    main()
