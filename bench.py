"""bench.py — aligned Gbases/s (PAF out) of the MI355X mapping path.

Workload (BASELINE.json metric): ONT-shaped 10 kb reads vs an hg38-shaped
synthetic reference (24 contigs with GRCh38 primary lengths, Σ≈3.1 Gb,
repeat families injected), index resident in HBM.  One step
= the whole hot path over one batch of reads already resident in HBM:
sketch -> query filter -> index lookup -> anchors -> sort -> chain DP
(+rescue) -> epilogue -> results to host -> PAF text.  Index build/upload
and mid_occ are outside the timed region.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py
--gpus N): one process per GPU, each with its own replicated index and its
own reads (weak scaling, no collective on the data path); barrier +
synchronize around the timed region, max-over-ranks time, value = all
ranks' bases / that time.

Output: ONE JSON line on rank 0 with the driver contract fields plus
"roofline" (dominant kernel, HIP events on the library stream) and
"cpu_baseline" (the C++ oracle restatement of the reference align on a
bounded sample of the same reads, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
HBM_COPY_GBS = 6290.0          # measured copy bandwidth (same guide)


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--reads", type=int, default=10000, help="reads per GPU per step (metric: 10k x 10 kb)")
    p.add_argument("--read-len", type=int, default=10000)
    p.add_argument("--scale", type=float, default=1.0, help="reference size relative to hg38 (1.0 = 3.1 Gb)")
    p.add_argument("--preset", default="hg38", choices=["hg38", "ecoli"],
                   help="synthetic reference: hg38-shaped (C3/C5 configs) or E. coli-shaped (C2)")
    p.add_argument("--ref-seed", type=int, default=38)
    p.add_argument("--read-seed", type=int, default=3)
    p.add_argument("--threads", type=int, default=0, help="host threads for index build (0 = auto)")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample duration")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    p.add_argument("--host-index", action="store_true", help="build the index on the host instead of the GPU")
    p.add_argument("--stats", default="", help="write per-read chain statistics (npz) to this path")
    p.add_argument("--streams", type=int, default=2,
                   help="contexts (HIP streams) per GPU, each mapping a contiguous share of the step's reads "
                        "from its own host thread against one shared device index")
    return p.parse_args()


def share_cuts(n: int, s: int):
    """Contiguous shares of n reads for s contexts: [cuts[k], cuts[k+1])."""
    s = max(1, s)
    return [round(k * n / s) for k in range(s + 1)]


def rank_read_seed(read_seed: int, rank: int) -> int:
    """Weak scaling: every rank maps its own reads (no data-path collective)."""
    return read_seed + rank


def reduce_step_time(dist, elapsed: float, n_bases: int, world: int, device):
    """Max-over-ranks wall time and all ranks' bases (one all-reduce each,
    outside the timed region)."""
    if world <= 1:
        return elapsed, float(n_bases)
    import torch
    tt = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    bt = torch.tensor([float(n_bases)], dtype=torch.float64, device=device)
    dist.all_reduce(bt, op=dist.ReduceOp.SUM)
    return float(tt.item()), float(bt.item())


SORT_SMALL = 4096   # reads up to this many anchors are sorted by k_sort_small (mm2g_kernels.hip)


def bench_config_tag(args) -> str:
    return f"reads={args.reads},read_len={args.read_len},streams={max(1, args.streams)},scale={args.scale}"


def pmc_traffic(kernel: str, tag: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC
    passes (profiles/pmc_traffic.json, written by tools/pmc_traffic.py:
    2 x FETCH_SIZE + WRITE_SIZE, the gfx950 correction of
    MI355X_MICROARCH.md §HBM) when they were taken with this bench
    configuration; otherwise None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as fh:
            t = json.load(fh)
        if t.get("bench_config") != tag:
            return None
        return t["kernels"][kernel]["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def host_threads(world: int) -> int:
    n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if n <= 0:
        try:
            n = len(os.sched_getaffinity(0))
        except AttributeError:
            n = os.cpu_count() or 8
    return max(1, min(n, 64) // max(world, 1))


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")

    import torch
    import torch.distributed as dist

    # one process per GPU; MM2G_DIST_BACKEND=gloo rehearses the launch on fewer GPUs
    backend = os.environ.get("MM2G_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    gpu = local % max(ndev, 1)
    if world > 1:
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    red_dev = "cuda" if backend == "nccl" else "cpu"

    import minimap2_rs_amd as M
    from minimap2_rs_amd import _lib as L
    from tools import simdata

    lib = L.load()                               # libmm2g.so (fails loudly if missing)
    if lib.mm2g_device_count() <= 0:
        raise SystemExit("bench.py: no HIP device visible")
    thr = args.threads or host_threads(world)

    # ---- reference + index (outside the timed region) ----------------------
    t0 = time.time()
    names, lens, gbuf = simdata.genome(args.preset, args.scale, args.ref_seed, threads=thr)
    log(f"rank {rank}: reference {lens.sum() / 1e9:.3f} Gb, {len(lens)} contigs in {time.time() - t0:.1f}s")
    t0 = time.time()
    # GPU index build (byte-identical to the host build, tests/test_gpu_parity.py)
    idx = M.Index.build_from_buffer(names, gbuf, lens, w=10, k=15, b=14, flag=0, threads=thr,
                                    device=None if args.host_index else gpu)
    t_index = time.time() - t0
    t0 = time.time()
    mid_host = idx.calc_mid_occ(2e-4)            # the reference's sort of all counts (index.rs:124-141)
    t_mid_host = time.time() - t0
    log(f"rank {rank}: index built ({'host' if args.host_index else 'GPU'}) in {t_index:.1f}s, stats {idx.stats()}")

    # ---- reads (per rank: distinct seed) -----------------------------------
    rbuf, roffs, _ = simdata.reads(gbuf, lens, args.reads, args.read_len, rank_read_seed(args.read_seed, rank))
    rnames = [f"r{i}" for i in range(args.reads)]
    n_bases = int(roffs[-1])

    S = max(1, args.streams)
    devs = [M.Device(gpu) for _ in range(S)]
    t0 = time.time()
    devs[0].upload_index(idx, 10)
    t_up = time.time() - t0
    # mid_occ from the device table's count histogram, checked against the host's
    t0 = time.time()
    mid_dev = devs[0].index_mid_occ(2e-4)
    t_mid_dev = time.time() - t0
    if mid_dev != mid_host:
        raise SystemExit(f"bench.py: device mid_occ {mid_dev} != host {mid_host}")
    mid = max(mid_dev, 10)                       # main.rs:196-197
    devs[0].set_mid_occ(mid)
    for d in devs[1:]:
        d.share_index(devs[0], mid)
    log(f"rank {rank}: mid_occ {mid} (device {t_mid_dev * 1e3:.1f} ms, host sort {t_mid_host * 1e3:.0f} ms)")
    # contiguous shares of the batch, one per context; reads resident in HBM before timing
    cuts = share_cuts(args.reads, S)
    shards = []
    t0 = time.time()
    for k, d in enumerate(devs):
        lo_r, hi_r = cuts[k], cuts[k + 1]
        sub_offs = (roffs[lo_r:hi_r + 1] - roffs[lo_r]).astype(np.uint64)
        d.set_reads_packed(rbuf[int(roffs[lo_r]):int(roffs[hi_r])], sub_offs)
        nr = hi_r - lo_r
        shards.append({
            "dev": d, "n": nr,
            "res": (L.ReadResult * max(nr, 1))(),
            "names": (C.c_char_p * max(nr, 1))(*[x.encode() for x in rnames[lo_r:hi_r]]),
            "cap": 256 * nr + (1 << 20),
        })
        shards[-1]["buf"] = C.create_string_buffer(shards[-1]["cap"])
        shards[-1]["len"] = 0
    t_h2d = time.time() - t0
    log(f"rank {rank}: index upload {t_up:.1f}s ({S} contexts share it), reads H2D {t_h2d * 1e3:.1f} ms ({n_bases / 1e9:.3f} Gb)")

    opts = M.map_opts()
    ih = idx._h

    def run_shard(sh):
        h = sh["dev"]._h
        L.check(lib.mm2g_batch_map(h, C.byref(opts)), "batch_map")
        L.check(lib.mm2g_batch_results(h, sh["res"], sh["n"]), "batch_results")
        sh["len"] = L.check(lib.mm2g_format_paf(ih, sh["res"], sh["names"], sh["n"], sh["buf"], sh["cap"]), "format_paf")

    import concurrent.futures as cf
    pool = cf.ThreadPoolExecutor(max_workers=S) if S > 1 else None

    def step() -> int:
        if pool is None:
            run_shard(shards[0])
        else:
            for f in [pool.submit(run_shard, sh) for sh in shards]:
                f.result()
        return sum(sh["len"] for sh in shards)

    for _ in range(args.warmup):
        step()
    paf_len = step() if args.warmup == 0 else None

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for d in devs:
        d.prof_enable(True)
        d.prof_reset()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        paf_len = step()
    barrier()
    elapsed = time.perf_counter() - t0
    prof = {}
    cnt = {}
    for d in devs:
        for k, (ms, calls) in d.prof().items():
            a0, c0 = prof.get(k, (0.0, 0))
            prof[k] = (a0 + ms, c0 + calls)
        d.prof_enable(False)
        for k, v in d.counters().items():        # per batch (identical every step)
            cnt[k] = cnt.get(k, 0) + v
    paf_all = b"".join(sh["buf"].raw[:sh["len"]] for sh in shards)
    if args.stats:
        cs = np.concatenate([d.chain_stats() for d in devs])
        na = np.array([sh["res"][i].n_anchors for sh in shards for i in range(sh["n"])], dtype=np.int64)
        fl = np.array([sh["res"][i].flags for sh in shards for i in range(sh["n"])], dtype=np.int64)
        np.savez(args.stats, chain=cs, n_anchors=na, flags=fl)

    elapsed, all_bases = reduce_step_time(dist, elapsed, n_bases, world, red_dev)
    total_bases = all_bases * args.steps

    value = total_bases / elapsed / 1e9
    ms_per_step = elapsed / max(args.steps, 1) * 1e3
    n_lines = paf_all.count(b"\n")

    # ---- roofline of the dominant kernel (HIP events on the library stream) --
    # Algorithmic bytes per launch (DESIGN.md "Roofline accounting").
    A, Ar, m, mk = cnt["anchors"], cnt["rescued_anchors"], cnt["minimizers"], cnt["kept_minimizers"]
    L_tot = cnt["bases"]
    na = np.array([sh["res"][i].n_anchors for sh in shards for i in range(sh["n"])], dtype=np.int64)
    A_large = int(na[na > SORT_SMALL].sum())
    A_small = int(na[(na > 1) & (na <= SORT_SMALL)].sum())
    kernel_bytes = {   # slot -> (kernel symbol, algorithmic bytes per step)
        "sketch": ("k_sketch", L_tot + 12 * m),              # ASCII in; (x 8 B, y 4 B) per minimizer out
        "filter": ("k_filter", 9 * m),                       # x in, keep flag out
        "seed_count": ("k_seed_count", 9 * m + 16 * mk + 8 * m),   # keep+x in, 16 B table entry per kept, (n, poff) out
        "seed_write": ("k_seed_write", 12 * m + 16 * A),     # (n, poff, y) in; 8 B position in + 8 B key out per anchor
        "sort_small": ("k_sort_small", 16 * A_small),        # each 8 B key read once and written once
        "sort_large": ("k_sort_read", 16 * A_large),
        "chain_seg": ("k_chain_seg", 8 * A),                 # every key read once (segmenting)
        "dv": ("k_dv", 0),
    }
    per_kernel = {}
    for name, (ms, calls) in prof.items():
        if calls > 0:
            per_kernel[name] = {"ms_per_step": ms / args.steps, "launches_per_step": calls / args.steps}
    cand = {k: v for k, v in prof.items() if k in kernel_bytes and kernel_bytes[k][1] > 0 and v[1] > 0}
    dom = max(cand, key=lambda k: cand[k][0])
    d_ms, d_calls = cand[dom]
    d_sym, d_bytes = kernel_bytes[dom]
    avg_s = d_ms / 1e3 / max(d_calls, 1)
    bytes_per_launch = d_bytes * args.steps / max(d_calls, 1)
    achieved = bytes_per_launch / avg_s / 1e9 if avg_s > 0 else 0.0
    traffic = pmc_traffic(d_sym, bench_config_tag(args))
    roofline = {
        "bound": "hbm", "kernel": d_sym, "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
        "avg_launch_ms": round(avg_s * 1e3, 4), "alg_bytes_per_launch": int(bytes_per_launch),
    }
    # whole-path algorithmic bytes (SURVEY.md §8d B(read) summed) over the step time
    B_path = (L_tot + 3) // 4 + 16 * mk + 48 * A + 24 * Ar
    path_gbs = B_path * args.steps / elapsed / 1e9 if world == 1 else None
    dp_pairs_s = cnt["dp_pairs"] * args.steps / elapsed if world == 1 else None

    # ---- CPU baseline: the oracle restatement on a bounded sample (rank 0, N=1) ---
    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu, parity = cpu_baseline(args, names, lens, gbuf, rbuf, roffs, rnames, mid, thr, paf_all)

    if rank == 0:
        line = {
            "metric": "aligned Gbases/sec (PAF out), 10k×10kb ONT reads vs hg38, 1/2/4/8 GPUs",
            "value": round(value, 6),
            "unit": "Gbases/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (hg38-shaped reference, seeded ONT-shaped reads; SURVEY.md §8d)",
            "config": {
                "workload": f"{args.preset}-shaped {lens.sum() / 1e9:.2f} Gb reference index in HBM + "
                            f"{args.reads}x{args.read_len // 1000} kb ONT reads per GPU per step",
                "reads_per_gpu_step": args.reads, "read_len": args.read_len, "ref_bases": int(lens.sum()),
                "mid_occ": mid, "parallelism": f"reads sharded x{world} (index replicated), {S} streams per GPU",
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
            "extra": {
                "paf_lines_per_step": n_lines,
                "per_kernel": per_kernel,
                "counters_per_step": cnt,
                "path_alg_GBps": round(path_gbs, 3) if path_gbs else None,
                "path_frac_of_8TBps": round(path_gbs / HBM_PEAK_GBS, 6) if path_gbs else None,
                "dp_pairs_per_s": dp_pairs_s,
                "index_build_s": round(t_index, 3), "index_build_on": "host" if args.host_index else "gpu",
                "index_upload_s": round(t_up, 3),
                "mid_occ_device_ms": round(t_mid_dev * 1e3, 2), "mid_occ_host_sort_ms": round(t_mid_host * 1e3, 1),
                "reads_h2d_ms": round(t_h2d * 1e3, 3),
                "pcie_inclusive_gbases_s": round(n_bases / (ms_per_step / 1e3 + t_h2d) / 1e9, 6) if world == 1 else None,
                "parity_vs_oracle": parity,
            },
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(args, names, lens, gbuf, rbuf, roffs, rnames, mid, thr, gpu_paf: bytes):
    """Time oracle/ (the C++ restatement of the reference align, 1 thread) on
    the first reads of the same batch; check its PAF against the GPU's."""
    from oracle import oracle as O
    import tempfile

    O.set_quiet(True)
    t0 = time.time()
    oi = O.OIndex.build_from_buffer(names, gbuf, lens, w=10, k=15, b=14, flag=0, threads=thr)
    log(f"oracle index built in {time.time() - t0:.1f}s")
    # calibrate on a few reads, then size the sample to ~cpu_seconds
    n_cal = min(10, args.reads)
    _, _, t_cal = oi.align_buffer(rnames[:n_cal], rbuf, roffs[: n_cal + 1], None, mid_occ=mid, threads=1)
    per_read = max(t_cal / n_cal, 1e-4)
    n_s = int(min(args.reads, max(n_cal, args.cpu_seconds / per_read)))
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "cpu.paf")
        n_lines, counts, t1 = oi.align_buffer(rnames[:n_s], rbuf, roffs[: n_s + 1], out, mid_occ=mid, threads=1)
        cpu_lines = open(out, "rb").read().splitlines()
    bases = int(roffs[n_s] - roffs[0])
    v1 = bases / t1 / 1e9
    # all-cores variant (OpenMP-style dynamic over reads): same sample
    _, _, tN = oi.align_buffer(rnames[:n_s], rbuf, roffs[: n_s + 1], None, mid_occ=mid, threads=thr)
    vN = bases / tN / 1e9
    log(f"cpu baseline: {n_s} reads, 1 thread {t1:.1f}s ({v1 * 1e3:.3f} Mb/s); {thr} threads {tN:.1f}s")
    # parity: GPU PAF lines for the sampled reads vs the oracle's
    want = set(rnames[:n_s])
    gpu_lines = [ln for ln in gpu_paf.splitlines() if ln.split(b"\t", 1)[0].decode() in want]
    parity = {"reads": n_s, "gpu_lines": len(gpu_lines), "cpu_lines": len(cpu_lines),
              "identical": gpu_lines == cpu_lines, "cpu_panics": counts.get("panics")}
    oi.close()
    cpu = {"value": round(v1, 9), "unit": "Gbases/s", "cores": 1, "kind": "port",
           "sample": f"first {n_s} of the step's {args.reads} reads ({bases / 1e6:.1f} Mb), oracle/ C++ restatement "
                     f"of mm2rs align, 1 thread, index build excluded",
           "all_cores": {"value": round(vN, 9), "cores": thr}}
    return cpu, parity


if __name__ == "__main__":
    main()
