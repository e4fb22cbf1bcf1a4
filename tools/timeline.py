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
    # busy fraction per tenth of the window: the warm-up, the ramp at the start of
    # the timed region and the isolated runs after it show as dips; the steady
    # state of the timed region is the plateau
    marks = sorted([(s, 1) for s, e, n in rows] + [(e, -1) for s, e, n in rows])
    edges = [t0 + (win * k) // 10 for k in range(11)]
    sl = [0] * 10
    live, prev = 0, t0
    for t, d in marks + [(t1, 0)]:
        if live > 0:
            a = prev
            while a < t:
                k = min(9, (a - t0) * 10 // win)
                b = min(t, edges[k + 1])
                sl[k] += b - a
                a = b if b > a else t
        prev = t
        live += d
    print("busy per tenth of the window: " + " ".join(f"{x / (win / 10):.2f}" for x in sl))


if __name__ == "__main__":
    main()
