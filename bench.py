"""bench.py — aligned Gbases/s (PAF out) of the MI355X mapping path.

Workload (BASELINE.json metric, config C3 of SURVEY.md §8d): ONT-shaped
10 kb reads vs an hg38-shaped synthetic reference (24 contigs with GRCh38
primary lengths, Σ≈3.1 Gb, repeat families injected), index resident in HBM.

One step = one batch of 10k distinct reads per GPU taken from reads
resident in host RAM (ASCII, as a FASTA reader leaves them) to all PAF lines
written, exactly as SURVEY.md §8d times it:
  nt4 2-bit packing on host threads into pinned memory -> H2D ->
  sketch -> query filter -> index lookup -> anchors -> sort -> chain DP
  (+rescue) -> epilogue -> per-read results to host -> PAF text.
Every step maps a different batch (a pool of W+K batches is generated up
front; the metric's 100k-read C3 set is 10 such batches).  Each batch is
cut into `--shares P` units (default 2); `--streams S` contexts per GPU
(default 4; own HIP stream and host thread each, one shared device index)
pull units from one queue, so the GPU always has queued units while other
contexts pack reads or format PAF.  Index build/upload and
mid_occ are outside the timed region.  The rate with reads already resident
in HBM is reported in `extra`.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py
--gpus N, or plain `python bench.py --gpus N`, which starts the N rank
processes itself before anything touches a GPU): one process per GPU with its
own reads (weak scaling, no collective on the data path); rank 0 generates
the reference once and shares it through /dev/shm, builds the index once and
the other ranks load its .mmi from there; barrier + synchronize around the
timed region, max-over-ranks time, value = all ranks' bases / that time; a
sample of every rank's reads is checked against the oracle on rank 0.  A
rank count that does not match --gpus, or more RCCL ranks than visible GPUs,
is an error, never a silent 1-GPU run.

Output: ONE JSON line on rank 0 with the driver contract fields plus
"roofline" (dominant kernel, HIP events on the library stream) and
"cpu_baseline" (the C++ oracle restatement of the reference align on a
bounded sample of the same reads, rank 0 at N=1 only, median of 3).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import ctypes as C
import hashlib
import json
import os
import socket
import statistics
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
HBM_COPY_GBS = 6290.0          # measured copy bandwidth (same guide)
VALU_INT32_OPS = 7.9e13        # 256 CU x 128 lanes/clk x 2.4 GHz
OPS_PER_PAIR = 15              # int32 ops per DP pair evaluation
SORT_CELL_MAX = 65535          # reads with more anchors take the large-read sort (k_sort_big)
SORT_SMALL = 4096              # reads up to this many anchors are sorted by k_sort_small (mm2g_kernels.hip)

# numpy view of mm2g_read_result (include/mm2g.h, 72 B)
RES_DTYPE = np.dtype([("flags", "<i4"), ("n_anchors", "<i4"), ("score", "<i4"), ("cm", "<i4"), ("qs", "<i4"), ("qe", "<i4"),
                      ("ts", "<i4"), ("te", "<i4"), ("rid", "<i4"), ("rev", "<i4"), ("n_match", "<i4"), ("dv_st", "<i4"),
                      ("dv_en", "<i4"), ("m_dv", "<i4"), ("sum_k", "<i8"), ("qlen", "<i4"), ("dv", "<f4")])
assert RES_DTYPE.itemsize == 72


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)    # the driver's own setting (BENCH_r05 "cmd")
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--reads", type=int, default=10000, help="reads per GPU per step (metric: 10k x 10 kb)")
    p.add_argument("--read-len", type=int, default=10000)
    p.add_argument("--scale", type=float, default=1.0, help="reference size relative to hg38 (1.0 = 3.1 Gb)")
    p.add_argument("--preset", default="hg38", choices=["hg38", "ecoli"],
                   help="synthetic reference: hg38-shaped (C3/C5 configs) or E. coli-shaped (C2)")
    p.add_argument("--ref-seed", type=int, default=38)
    p.add_argument("--read-seed", type=int, default=3)
    p.add_argument("--max-batches", type=int, default=40, help="distinct read batches generated (steps cycle beyond)")
    p.add_argument("--threads", type=int, default=0, help="host threads for index build (0 = auto)")
    p.add_argument("--pack-threads", type=int, default=0, help="host threads per context packing reads to nt4 (0 = auto)")
    p.add_argument("--cpu-seconds", type=float, default=8.0, help="target duration of one CPU-baseline run (3 runs, median)")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline (parity sample still checked)")
    p.add_argument("--no-parity", action="store_true", help="skip the oracle parity check as well")
    p.add_argument("--host-index", action="store_true", help="build the index on the host instead of the GPU")
    p.add_argument("--resident-steps", type=int, default=3, help="extra: steps re-mapping reads already in HBM")
    p.add_argument("--knob", action="append", default=[], metavar="NAME=VALUE",
                   help="context knob for A/B runs (include/mm2g.h MM2G_KNOB_*), e.g. sort_prof=1")
    p.add_argument("--index-knob", action="append", default=[], metavar="NAME=VALUE",
                   help="process-wide index-build knob (include/mm2g.h MM2G_IKNOB_*), e.g. force_fallback=1")
    p.add_argument("--streams", type=int, default=6,
                   help="contexts (HIP streams) per GPU, each with its own host thread, sharing one device index "
                        "(round 6: 6 over 4 by +6.5 %% on C3 at 20 and 60 steps, +4 %% on C2 with one share, "
                        "even on C5: profiles/r06_ab/*streams*.txt)")
    p.add_argument("--shares", type=int, default=-1,
                   help="units each batch is cut into (0 = one per stream); contexts pull units from one queue; "
                        "-1 = auto: 1 for steps of <= 2000 reads (C2 +50 %%, C5 +9 %% in round 6), else 2 "
                        "(profiles/r06_ab/shares_*.txt)")
    p.add_argument("--min-cnt", type=int, default=3, help="-n (main.rs:45); <= 1 with --min-chain-score <= k: the multi-chain output")
    p.add_argument("--min-chain-score", type=int, default=40, help="-m (main.rs:48)")
    p.add_argument("--iso-batches", type=int, default=3,
                   help="batches mapped by one context after the timed region for the roofline's quiet-GPU launch times")
    args = p.parse_args(argv)
    if args.shares < 0:
        args.shares = 1 if args.reads <= 2000 else 2
    return args


def share_cuts(n: int, s: int):
    """Contiguous shares of n reads for s contexts: [cuts[k], cuts[k+1])."""
    s = max(1, s)
    return [round(k * n / s) for k in range(s + 1)]


def batch_seed(read_seed: int, rank: int, b: int) -> int:
    """Weak scaling: every rank maps its own reads, a distinct batch every step
    (rank 0's batch 0 is the §8d read seed itself)."""
    return read_seed + 1_000_003 * rank + 7_919 * b


def rank_read_seed(read_seed: int, rank: int) -> int:
    return batch_seed(read_seed, rank, 0)


def reduce_step_time(dist, elapsed: float, n_bases: int, world: int, device):
    """Max-over-ranks wall time, all ranks' bases and every rank's own time (an
    all-reduce each and one all-gather, outside the timed region): the per-rank
    times make a short multi-GPU line diagnosable (which rank, how uneven)."""
    if world <= 1:
        return elapsed, float(n_bases), [elapsed]
    import torch
    tt = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    bt = torch.tensor([float(n_bases)], dtype=torch.float64, device=device)
    dist.all_reduce(bt, op=dist.ReduceOp.SUM)
    every = [None] * world
    dist.all_gather_object(every, float(elapsed))
    return float(tt.item()), float(bt.item()), [float(x) for x in every]


def rank_times(every, steps: int) -> dict:
    """Per-rank ms/step and the straggler ratio max/mean over ranks."""
    ms = [x / max(steps, 1) * 1e3 for x in every]
    mean = sum(ms) / max(len(ms), 1)
    return {"per_rank_ms_per_step": [round(x, 3) for x in ms],
            "rank_time_max_over_mean": round(max(ms) / mean, 4) if mean > 0 else None}


def ref_size(nb: int) -> str:
    """Reference size for config.workload: Gb above 0.1 Gb, else Mb (E. coli is 4.64 Mb, not 0.00 Gb)."""
    return f"{nb / 1e9:.2f} Gb" if nb >= 1e8 else f"{nb / 1e6:.2f} Mb"


def affinity_cpus() -> int:
    """CPUs in this process's affinity set (the CPU baseline's all-cores leg uses every one)."""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def device_identity(gpu: int) -> str:
    """A stable name of the GPU this rank drives (UUID where torch exposes it)."""
    import torch
    try:
        pr = torch.cuda.get_device_properties(gpu)
        u = getattr(pr, "uuid", None)
        if u:
            return str(u)
        return f"{getattr(pr, 'pci_domain_id', '?')}:{getattr(pr, 'pci_bus_id', '?')}:{getattr(pr, 'pci_device_id', gpu)}"
    except Exception:
        return f"dev{gpu}"


def count_devices(dist, world: int, ident) -> int:
    """Distinct (host, device) pairs over the ranks: n_gpus counts GPUs, not ranks."""
    if world <= 1:
        return 1
    got = [None] * world
    dist.all_gather_object(got, (socket.gethostname(), ident))
    return len(set(got))


def rank_env(argv_gpus: int, env=None):
    """(rank, world, local_rank) from the launcher's environment, checked
    against --gpus: a mismatch is an error, never a silent smaller run."""
    env = os.environ if env is None else env
    world = int(env.get("WORLD_SIZE", "1"))
    rank = int(env.get("RANK", "0"))
    local = int(env.get("LOCAL_RANK", str(rank)))
    if world != argv_gpus:
        raise SystemExit(f"bench.py: --gpus {argv_gpus} but the launcher started WORLD_SIZE={world} ranks; "
                         f"run `python bench.py --gpus {argv_gpus}` (it starts the ranks itself) or "
                         f"`python -m torch.distributed.run --nproc-per-node {argv_gpus} bench.py --gpus {argv_gpus}`")
    return rank, world, local


def spawn_ranks(n: int, argv, backend: str, ndev: int, cmd=None) -> int:
    """`--gpus N` (N > 1) without a launcher: start the N rank processes of this
    script as fresh children (this process never touches a GPU, so nothing is
    exec'd from a GPU process), with the environment torch.distributed.run
    gives them, and wait (minimap2_rs_amd.shard.spawn_ranks).  Rank 0 prints the
    line.  One failing rank stops the others; the exit code is the first failure's."""
    if backend == "nccl" and ndev < n:
        raise SystemExit(f"bench.py: --gpus {n} needs {n} GPUs for {n} RCCL ranks, {ndev} visible "
                         f"(MM2G_DIST_BACKEND=gloo rehearses {n} ranks on fewer GPUs)")
    from minimap2_rs_amd.shard import spawn_ranks as spawn
    return spawn(n, list(cmd or [sys.executable, os.path.abspath(__file__)]) + list(argv), log=log)


def paf_lines_by_read(paf: bytes):
    """PAF text -> {read name: its lines} (one line per mapped read, SURVEY.md Q4;
    several, newline-joined in output order, under -n <= 1 -m <= k)."""
    out = {}
    for ln in paf.splitlines():
        nm = ln.split(b"\t", 1)[0].decode()
        out[nm] = out[nm] + b"\n" + ln if nm in out else ln
    return out


def kernel_sha() -> str:
    """Hash of the kernel sources: profiles/pmc_traffic.json is used only when
    its counters were taken on these exact kernels."""
    h = hashlib.sha256()
    for f in ("mm2g_kernels.hip", "mm2g_internal.h"):
        with open(os.path.join(ROOT, "minimap2_rs_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def bench_config_tag(args) -> str:
    tag = f"reads={args.reads},read_len={args.read_len},streams={max(1, args.streams)},shares={args.shares},scale={args.scale},preset={args.preset}"
    if (getattr(args, "min_cnt", 3), getattr(args, "min_chain_score", 40)) != (3, 40):
        tag += f",n={args.min_cnt},m={args.min_chain_score}"
    return tag


def pmc_traffic(kernel: str, hint: str, tag: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (profiles/pmc_traffic.json, tools/pmc_traffic.py: 2 x FETCH_SIZE +
    WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md §HBM) when they
    were taken with this bench configuration on these kernel sources; else
    None.  Template instantiations are separate rows: `hint` picks the one the
    mapping path runs (e.g. SeqNt4 for the query sketch).
    -> (bytes per launch, row name) or (None, None)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as fh:
            t = json.load(fh)
        if t.get("bench_config") != tag or t.get("kernels_sha") != kernel_sha():
            return None, None
        rows = {k: v for k, v in t["kernels"].items() if k.split("<")[0] == kernel}
        if len(rows) > 1 and hint:
            rows = {k: v for k, v in rows.items() if hint in k}
        if len(rows) != 1:
            return None, None
        (k, v), = rows.items()
        return v["hbm_bytes_per_launch"], k
    except (OSError, KeyError, ValueError):
        return None, None


def host_threads(world: int) -> int:
    n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if n <= 0:
        try:
            n = len(os.sched_getaffinity(0))
        except AttributeError:
            n = os.cpu_count() or 8
    return max(1, min(n, 64) // max(world, 1))


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def make_batches(gbuf, lens, args, rank, n_batches, threads):
    """n_batches distinct batches of reads (ASCII in host RAM), generated in parallel."""
    from tools import simdata

    def one(b):
        rb, offs, _ = simdata.reads(gbuf, lens, args.reads, args.read_len, batch_seed(args.read_seed, rank, b))
        return rb, offs
    with cf.ThreadPoolExecutor(max_workers=max(1, min(threads, 16))) as ex:
        return list(ex.map(one, range(n_batches)))


def shared_genome(args, dist, rank: int, world: int, thr: int, tag: str):
    """The synthetic reference.  With several ranks, rank 0 generates it once and
    shares it through /dev/shm (the others map the file read-only) instead of
    every rank regenerating 3.1 Gb; if /dev/shm has no room, each rank generates
    its own (the same seeded bytes)."""
    from tools import simdata
    if world <= 1:
        return simdata.genome(args.preset, args.scale, args.ref_seed, threads=thr)
    path = f"/dev/shm/mm2g_bench_{tag}.genome"
    meta = [None]
    gbuf = None
    if rank == 0:
        names, lens, gbuf = simdata.genome(args.preset, args.scale, args.ref_seed, threads=thr)
        ok = True
        try:
            gbuf.tofile(path)
        except OSError as e:
            log(f"rank 0: reference to {path} failed ({e}); every rank generates its own")
            ok = False
        meta = [(names, [int(x) for x in lens], ok)]
    dist.broadcast_object_list(meta, src=0)
    names, lens_l, ok = meta[0]
    lens = np.array(lens_l, dtype=np.int64)
    if rank != 0:
        if ok:
            gbuf = np.memmap(path, dtype=np.uint8, mode="r", shape=(int(lens.sum()),))
        else:
            names, lens, gbuf = simdata.genome(args.preset, args.scale, args.ref_seed, threads=thr)
    dist.barrier()
    if rank == 0 and ok:
        os.unlink(path)          # the ranks' mappings keep the pages until they exit
    return names, lens, gbuf


# slot (mm2g_prof name) -> (kernel symbol, instantiation hint for the PMC rows)
KERNEL_SYMBOLS = {
    "mz_base": ("k_mz_base", ""), "sketch": ("k_sketch", "SeqNt4"), "scan": ("k_excl_scan", ""),
    "filter": ("k_filter", ""), "seed_count": ("k_seed_count", ""), "seed_write": ("k_seed_write", ""),
    "sort_small": ("k_sort_small", ""), "sort_large": ("k_sort_read", ""), "sort_radix": ("k_sort_radix", ""),
    "sort_big": ("k_sort_big", ""),
    "chain_items": ("k_seg_items", ""), "chain_lb": ("k_chain_lb", ""), "chain_cands": ("k_seg_cands", ""),
    "chain_seg": ("k_chain_seg", ""),
    "chain_med": ("k_chain_med", ""), "chain_lorder": ("k_lseg_order", ""), "chain_long": ("k_chain_long", ""),
    "chain_giant": ("k_chain_giant", ""), "chain_fin": ("k_chain_fin", ""),
    "chain_items_rescue": ("k_seg_items", ""), "chain_lb_rescue": ("k_chain_lb", ""), "chain_cands_rescue": ("k_seg_cands", ""),
    "chain_seg_rescue": ("k_chain_seg", ""), "chain_med_rescue": ("k_chain_med", ""),
    "chain_lorder_rescue": ("k_lseg_order", ""), "chain_giant_rescue": ("k_chain_giant", ""),
    "chain_long_rescue": ("k_chain_long", ""), "chain_fin_rescue": ("k_chain_fin", ""), "dv": ("k_dv", ""),
}
CHAIN_SLOTS = {k for k in KERNEL_SYMBOLS if k.startswith("chain_")}


def alg_bytes(cnt: dict, res) -> dict:
    """Algorithmic HBM bytes of every kernel slot over the mapped batches
    (SURVEY.md §8d per-anchor terms).  cnt: summed
    mm2g_batch_counters, res: the per-read results (RES_DTYPE).
    Sorts are priced at 16 B per anchor (each key read once and written once),
    whatever passes an implementation makes; chain kernels at 8 B of key in and
    8 B of f/pprev out per anchor of the segments they process.
    Fused seeding (counters 16/17): k_sort_read makes the keys of the reads it
    sorts, so k_seed_write is charged only for the other reads, and the sort
    for those reads' minimizer records (12 B) and position fetches (8 B per
    anchor) on top of its 16 B: SURVEY.md §8d's per-anchor position fetch +
    anchor write + anchor read at 8-B keys.  The same for
    the reads over 65535 anchors that k_sort_big seeds (counters 21/22)."""
    n = len(res)
    A, m, mk, L = cnt["anchors"], cnt["minimizers"], cnt["kept_minimizers"], cnt["bases"]
    Af, mf = cnt.get("fused_anchors", 0), cnt.get("fused_minimizers", 0)
    Ab, mb = cnt.get("fused_big_anchors", 0), cnt.get("fused_big_minimizers", 0)   # ... made by k_sort_big
    Adp = cnt.get("dp_anchors", A)
    na = res["n_anchors"].astype(np.int64)
    mapped = (res["flags"] & 1) != 0
    cm = int(res["cm"][mapped].astype(np.int64).sum())
    # anchors per sort class as the library dispatched them (counters 18-20): without the
    # singleton filter (multi-chain output, debug) every read above the small class goes whole
    # to k_sort_radix and k_sort_read only lists it
    if "sort_whole_anchors" in cnt:
        s_small, s_cell, s_whole = (cnt.get(k, 0) for k in ("sort_small_anchors", "sort_cell_anchors", "sort_whole_anchors"))
    else:
        s_small = int(na[(na > 1) & (na <= SORT_SMALL)].sum())
        s_cell = int(na[(na > SORT_SMALL) & (na <= SORT_CELL_MAX)].sum())
        s_whole = int(na[na > SORT_CELL_MAX].sum())
    mdv = int(res["m_dv"][mapped].astype(np.int64).sum())
    return {
        "mz_base": 24 * n,
        "sketch": (L + 3) // 4 + 12 * m,                 # nt4 codes in; (x 8 B, y 4 B) per minimizer out
        "scan": 24 * n,                                   # two scans: u32 in, u64 out per read
        "filter": 9 * m,                                  # x in, keep flag out
        "seed_count": 9 * m + 16 * mk + 8 * m,            # keep+x in, 16 B table entry per kept, (n, poff) out
        "seed_write": 12 * (m - mf - mb) + 16 * (A - Af - Ab),   # (n, poff, y) in; 8 B position in + 8 B key out per anchor
        "sort_small": 16 * s_small,
        "sort_large": 16 * s_cell + 12 * mf + 8 * Af,
        "sort_radix": 16 * s_whole,
        "sort_big": 16 * s_whole + 12 * mb + 8 * Ab,
        "chain_items": 8 * n,
        "chain_lb": 8 * cnt.get("lb_stream_anchors", Adp) + Adp // 8,   # keys in, segment-start bits out
        "chain_cands": Adp // 8 + 12 * n,                        # segment-start bits in (per read: a_off, cnt2, fmin)
        "chain_seg": 8 * cnt.get("seg_stream_anchors", Adp),    # the items left to streaming
        "chain_med": 16 * cnt.get("med_anchors", 0),
        "chain_lorder": 0,
        "chain_long": 16 * cnt.get("long_anchors", 0),
        "chain_giant": 16 * cnt.get("giant_anchors", 0),
        "chain_fin": 96 * n + 8 * cm,
        "chain_items_rescue": 8 * n,
        "chain_lb_rescue": 8 * cnt["rescued_anchors"] + cnt["rescued_anchors"] // 8,
        "chain_cands_rescue": cnt["rescued_anchors"] // 8 + 12 * n,
        "chain_seg_rescue": 8 * cnt.get("seg_stream_rescue", cnt["rescued_anchors"]),
        "chain_med_rescue": 16 * cnt.get("med_anchors_rescue", 0),
        "chain_lorder_rescue": 0,
        "chain_giant_rescue": 16 * cnt.get("giant_anchors_rescue", 0),
        "chain_long_rescue": 16 * cnt.get("long_anchors_rescue", 0),
        "chain_fin_rescue": 96 * n,
        "dv": 8 * cm + 4 * mdv,
    }


def main():
    args = parse()
    backend = os.environ.get("MM2G_DIST_BACKEND", "nccl")   # gloo: rehearse more ranks than GPUs
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        import torch
        ndev = torch.cuda.device_count()       # counts devices without initialising HIP on this image
        raise SystemExit(spawn_ranks(args.gpus, sys.argv[1:], backend, ndev))
    rank, world, local = rank_env(args.gpus)

    import torch
    import torch.distributed as dist

    ndev = torch.cuda.device_count()
    if backend == "nccl" and world > max(ndev, 1) and ndev >= 1:
        raise SystemExit(f"bench.py: {world} RCCL ranks but {ndev} GPU(s) visible: one rank per GPU "
                         f"(MM2G_DIST_BACKEND=gloo rehearses more ranks than GPUs)")
    gpu = local % max(ndev, 1)
    coll_seen = None
    if world > 1:
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    red_dev = "cuda" if backend == "nccl" else "cpu"
    if world > 1:
        one = torch.ones(1, dtype=torch.float64, device=red_dev)
        dist.all_reduce(one)                  # the ranks the collective backend actually joined
        coll_seen = int(one.item())
        if coll_seen != world:
            raise SystemExit(f"bench.py: {dist.get_backend()} all-reduce saw {coll_seen} ranks, expected {world}")

    import minimap2_rs_amd as M
    from minimap2_rs_amd import _lib as L

    lib = L.load()                               # libmm2g.so (fails loudly if missing)
    if lib.mm2g_device_count() <= 0:
        raise SystemExit("bench.py: no HIP device visible")
    thr = args.threads or host_threads(world)
    for kv in args.index_knob:
        k, v = kv.split("=", 1)
        M.set_index_knob(k, int(v))
    ident = device_identity(gpu)
    n_gpus = count_devices(dist, world, ident)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # ---- reference, read batches, index (outside the timed region) ----------
    tag = os.environ.get("MASTER_PORT", "0")
    t0 = time.time()
    names, lens, gbuf = shared_genome(args, dist, rank, world, thr, tag)
    log(f"rank {rank}: reference {lens.sum() / 1e9:.3f} Gb, {len(lens)} contigs in {time.time() - t0:.1f}s")
    # warmup: W steps, and at least one unit per context (each context's first
    # unit allocates its workspaces; with W * P < S some would pay that in the timed region)
    S_ctx = max(1, args.streams)
    w_eff = max(args.warmup, -(-S_ctx // (args.shares if args.shares > 0 else S_ctx)))
    n_batches = max(1, min(w_eff + args.steps, args.max_batches))
    t0 = time.time()
    batches = make_batches(gbuf, lens, args, rank, n_batches, thr)
    bases_per_batch = [int(b[1][-1]) for b in batches]
    log(f"rank {rank}: {n_batches} batches x {args.reads} reads generated in {time.time() - t0:.1f}s")
    t0 = time.time()
    idx = None
    shm = f"/dev/shm/mm2g_bench_{tag}.mmi"
    if rank == 0 or world == 1:
        # GPU index build (byte-identical to the oracle's, tests/test_gpu_parity.py)
        idx = M.Index.build_from_buffer(names, gbuf, lens, w=10, k=15, b=14, flag=0, threads=thr,
                                        device=None if args.host_index else gpu)
    if world > 1:
        ok = False
        if rank == 0:
            try:
                idx.save_to_mmi(shm)
                ok = True
            except Exception as e:   # no room in /dev/shm: every rank builds its own
                log(f"rank 0: .mmi to {shm} failed ({e}); ranks build their own index")
        flag = [ok]
        dist.broadcast_object_list(flag, src=0)
        if rank != 0:
            if flag[0]:
                idx = M.Index.load_from_mmi(shm)        # mapped, bucket-parallel load
            else:
                idx = M.Index.build_from_buffer(names, gbuf, lens, w=10, k=15, b=14, flag=0, threads=thr,
                                                device=None if args.host_index else gpu)
        dist.barrier()
        if rank == 0 and ok:
            os.unlink(shm)
    index_from, index_note = idx.origin               # what actually happened (mm2g_index_origin)
    t_index = time.time() - t0
    t0 = time.time()
    mid_host = idx.calc_mid_occ(2e-4)            # the reference's sort of all counts (index.rs:124-141)
    t_mid_host = time.time() - t0
    log(f"rank {rank}: index from {index_from}{' (' + index_note + ')' if index_note else ''} in {t_index:.1f}s, stats {idx.stats()}")

    S = max(1, args.streams)
    devs = [M.Device(gpu) for _ in range(S)]
    pack_thr = args.pack_threads or max(1, min(8, thr // S))
    for d in devs:
        d.set_knob("host_threads", pack_thr)
        for kv in args.knob:
            k, v = kv.split("=", 1)
            d.set_knob(k, int(v))
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
    idx.release_tables()                         # the device copy is made: keep only names/lengths on the host
    log(f"rank {rank}: index upload {t_up:.1f}s ({S} contexts share it), mid_occ {mid} "
        f"(device {t_mid_dev * 1e3:.1f} ms, host sort {t_mid_host * 1e3:.0f} ms)")

    opts = M.map_opts(min_cnt=args.min_cnt, min_chain_score=args.min_chain_score)
    multi = args.min_cnt <= 1 and args.min_chain_score <= 15   # the -n <= 1 -m <= k multi-chain output (k = 15)
    ih = idx._h
    P = args.shares if args.shares > 0 else S    # units per batch
    cuts = share_cuts(args.reads, P)
    # per (batch, share) unit: names, result array, PAF buffer
    units = []
    for b in range(n_batches):
        rb, offs = batches[b]
        for k in range(P):
            lo, hi = cuts[k], cuts[k + 1]
            nr = hi - lo
            sub = np.ascontiguousarray(offs[lo:hi + 1], dtype=np.uint64)     # absolute offsets into rb
            units.append({
                "b": b, "k": k, "lo": lo, "n": nr, "offs": sub,
                "names": (C.c_char_p * max(nr, 1))(*[read_name(rank, b, i).encode() for i in range(lo, hi)]),
                "res": (L.ReadResult * max(nr, 1))(),
                "cap": (1024 if multi else 256) * nr + (1 << 20), "len": 0, "cnt": None,
            })
            units[-1]["buf"] = C.create_string_buffer(units[-1]["cap"])

    def run_unit(d, u):
        h = d._h
        rb = batches[u["b"]][0]
        t = [time.perf_counter()]
        L.check(lib.mm2g_batch_set_reads(h, rb.ctypes.data_as(C.c_void_p), u["offs"].ctypes.data_as(L._P64), u["n"]), "set_reads")
        t.append(time.perf_counter())
        L.check(lib.mm2g_batch_map(h, C.byref(opts)), "batch_map")
        t.append(time.perf_counter())
        L.check(lib.mm2g_batch_results(h, u["res"], u["n"]), "batch_results")
        t.append(time.perf_counter())
        if multi:   # the host epilogue's several lines per read (mm2g_batch_paf)
            u["len"] = L.check(lib.mm2g_batch_paf(h, u["names"], u["n"], u["buf"], u["cap"]), "batch_paf")
        else:
            u["len"] = L.check(lib.mm2g_format_paf(ih, u["res"], u["names"], u["n"], u["buf"], u["cap"]), "format_paf")
        t.append(time.perf_counter())
        u["cnt"] = d.counters()
        u["host_ms"] = [(t[i + 1] - t[i]) * 1e3 for i in range(4)]

    def run_steps(s0: int, s1: int):
        """Map the units of steps [s0, s1) (step s -> batch s mod n_batches) on
        the S contexts, each pulling the next unit from a shared queue."""
        todo = [u for s in range(s0, s1) for u in units[(s % n_batches) * P:(s % n_batches + 1) * P]]
        nxt = [0]
        lock = threading.Lock()
        errs = []

        def worker(d):
            try:
                while True:
                    with lock:
                        i = nxt[0]
                        nxt[0] += 1
                    if i >= len(todo):
                        return
                    run_unit(d, todo[i])
            except Exception as e:   # surfaced after the join
                errs.append(e)
        ths = [threading.Thread(target=worker, args=(d,)) for d in devs]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        if errs:
            raise errs[0]

    run_steps(0, w_eff)
    for d in devs:
        d.prof_enable(True)
        d.prof_reset()
    barrier()
    t0 = time.perf_counter()
    run_steps(w_eff, w_eff + args.steps)
    barrier()
    elapsed = time.perf_counter() - t0
    prof = {}
    for d in devs:
        for k, (ms, calls) in d.prof().items():
            a0, c0 = prof.get(k, (0.0, 0))
            prof[k] = (a0 + ms, c0 + calls)
        d.prof_enable(False)
    timed = [units[(s % n_batches) * P + k] for s in range(w_eff, w_eff + args.steps) for k in range(P)]
    cnt = {}
    for u in timed:
        for k, v in u["cnt"].items():
            cnt[k] = cnt.get(k, 0) + v
    res_np = np.concatenate([np.frombuffer(u["res"], dtype=RES_DTYPE, count=u["n"]) for u in timed if u["n"]])
    n_lines = sum(bytes(u["buf"].raw[:u["len"]]).count(b"\n") for u in timed)
    # host-side time per unit (one share of one step): nt4 pack + H2D queue, map
    # queue, wait for results (incl. post-processing), PAF formatting
    hm = np.array([u["host_ms"] for u in timed])
    host_ms = dict(zip(("set_reads", "map_enqueue", "results_wait", "format_paf"), [round(float(x), 3) for x in hm.mean(axis=0)]))
    my_bases = sum(bases_per_batch[s % n_batches] for s in range(w_eff, w_eff + args.steps))

    # ---- extra: reads already resident in HBM (the round-1 headline) --------
    resident = None
    if args.resident_steps > 0 and P <= S:
        us = units[:P]
        for d, u in zip(devs, us):
            rb = batches[u["b"]][0]
            L.check(lib.mm2g_batch_set_reads(d._h, rb.ctypes.data_as(C.c_void_p), u["offs"].ctypes.data_as(L._P64), u["n"]), "set_reads")
            L.check(lib.mm2g_batch_map(d._h, C.byref(opts)), "batch_map")
            L.check(lib.mm2g_batch_results(d._h, u["res"], u["n"]), "batch_results")

        def resident_share(d, u):
            for _ in range(args.resident_steps):
                L.check(lib.mm2g_batch_map(d._h, C.byref(opts)), "batch_map")
                L.check(lib.mm2g_batch_results(d._h, u["res"], u["n"]), "batch_results")
                if multi:
                    L.check(lib.mm2g_batch_paf(d._h, u["names"], u["n"], u["buf"], u["cap"]), "batch_paf")
                else:
                    L.check(lib.mm2g_format_paf(ih, u["res"], u["names"], u["n"], u["buf"], u["cap"]), "format_paf")
        barrier()
        tr = time.perf_counter()
        ths = [threading.Thread(target=resident_share, args=(d, u)) for d, u in zip(devs, us)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        barrier()
        trs = time.perf_counter() - tr
        resident = {"gbases_s_per_gpu": round(bases_per_batch[0] * args.resident_steps / trs / 1e9, 6),
                    "ms_per_step": round(trs / args.resident_steps * 1e3, 3),
                    "note": "the same batch re-mapped from HBM: no host packing, no H2D (not the metric)"}

    elapsed, all_bases, every_rank = reduce_step_time(dist, elapsed, my_bases, world, red_dev)
    value = all_bases / elapsed / 1e9
    ms_per_step = elapsed / max(args.steps, 1) * 1e3

    # ---- roofline of the dominant kernel (HIP events on the library streams; roofline_of) --
    # every kernel slot is priced (alg_bytes); per_kernel holds the timed region's in-situ figures
    kb = alg_bytes(cnt, res_np)
    per_kernel = {}
    for name, (ms, calls) in prof.items():
        if calls > 0:
            b = kb.get(name)
            avg_s = ms / 1e3 / calls
            e = {"ms_per_step": round(ms / args.steps, 4), "launches_per_step": calls / args.steps}
            if b is not None and avg_s > 0:
                e["alg_GBps"] = round(b / calls / avg_s / 1e9, 2)
                e["hbm_frac"] = round(b / calls / avg_s / 1e9 / HBM_PEAK_GBS, 5)
            per_kernel[name] = e
    timed_slots = {k: v for k, v in prof.items() if v[1] > 0}
    chain_ms = sum(v[0] for k, v in timed_slots.items() if k in CHAIN_SLOTS)
    # the roofline is rank 0's (only rank 0 prints); the other ranks go straight to the parity gather
    roofline = iso = None
    fatal = []
    if rank == 0:
        roofline, iso, fatal = roofline_of(args, lib, L, devs, units, batches, P, opts, n_batches, cnt, kb, prof,
                                           timed_slots, chain_ms, per_kernel, ms_per_step, elapsed, world)
    # whole-path algorithmic bytes (SURVEY.md §8d B(read) summed) over the step time
    A, Ar, mk, L_tot = cnt["anchors"], cnt["rescued_anchors"], cnt["kept_minimizers"], cnt["bases"]
    B_path = (L_tot + 3) // 4 + 16 * mk + 48 * A + 24 * Ar
    path_gbs = B_path / elapsed / 1e9 if world == 1 else None
    dp_pairs_s = cnt["dp_pairs"] / elapsed if world == 1 else None

    # ---- oracle parity on a sample of every rank's timed batches; CPU baseline
    # N=1: ~3,000 reads (the CPU baseline's ~8 s runs come out of it); N>1: 500 per rank
    n_sample = 0 if args.no_parity else min(args.reads * args.steps, 3000 if world == 1 else 500)
    samp = sample_reads(args, batches, timed, n_sample, S, rank)
    gathered = [samp] if world == 1 else [None] * world
    if world > 1:
        dist.all_gather_object(gathered, samp)
    cpu = parity = None
    if rank == 0 and n_sample:
        cpu, parity = oracle_check(args, names, lens, gbuf, mid, thr, gathered, world)

    if fatal:   # after the gather (the other ranks are not left waiting in it)
        raise SystemExit("bench.py: " + "; ".join(fatal))
    if rank == 0:
        line = {
            "metric": "aligned Gbases/sec (PAF out), 10k×10kb ONT reads vs hg38, 1/2/4/8 GPUs",
            "value": round(value, 6),
            "unit": "Gbases/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (hg38-shaped reference, seeded ONT-shaped reads, a distinct batch every step; SURVEY.md §8d)",
            "config": {
                "workload": f"{args.preset}-shaped {ref_size(int(lens.sum()))} reference index in HBM + "
                            f"{args.reads}x{args.read_len // 1000} kb ONT reads per GPU per step, from host RAM "
                            f"(nt4 pack + H2D + map + PAF in the timed region)",
                "reads_per_gpu_step": args.reads, "read_len": args.read_len, "ref_bases": int(lens.sum()),
                "chain_opts": f"-n {args.min_cnt} -m {args.min_chain_score}" + (" (multi-chain output: device map with full DP "
                              "arrays, host backtrack/merge/select, mm2g_batch_paf)" if multi else ""),
                "distinct_batches": n_batches, "mid_occ": mid,
                "ranks": world, "distinct_devices": n_gpus,
                "collective_backend": (dist.get_backend() if world > 1 else None),
                "collective_world_seen": coll_seen if world > 1 else 1,
                "launch": ("self-spawned ranks" if os.environ.get("MM2G_BENCH_SPAWNED") else
                           ("torch.distributed.run" if world > 1 else "single process")),
                "parallelism": f"reads sharded x{world} (index replicated), {S} streams per GPU, {P} units per batch",
                **rank_times(every_rank, args.steps),
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
            "extra": {
                "paf_lines_per_step": n_lines / args.steps,
                "per_kernel": per_kernel,
                "counters_per_step": {k: v / args.steps for k, v in cnt.items()},
                "resident_in_hbm": resident,
                "quiet_gpu": iso,
                "path_alg_GBps": round(path_gbs, 3) if path_gbs else None,
                "path_frac_of_8TBps": round(path_gbs / HBM_PEAK_GBS, 6) if path_gbs else None,
                "dp_pairs_per_s": dp_pairs_s,
                "index_build_s": round(t_index, 3), "index_from": index_from, "index_fallback_reason": index_note,
                "index_upload_s": round(t_up, 3),
                "mid_occ_device_ms": round(t_mid_dev * 1e3, 2), "mid_occ_host_sort_ms": round(t_mid_host * 1e3, 1),
                "pack_threads_per_context": pack_thr,
                "host_ms_per_unit": host_ms,
                "parity_vs_oracle": parity,
            },
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def roofline_of(args, lib, L, devs, units, batches, P, opts, n_batches, cnt, kb, prof, timed_slots, chain_ms, per_kernel,
                ms_per_step, elapsed, world):
    """Rank 0: the roofline of the dominant kernel, from the same kernels on a quiet GPU.
    In the timed region four contexts' kernels share the GPU, so a launch's duration
    there includes the other contexts' work (a kernel's in-situ time per step can
    exceed the step).  The headline `frac` therefore comes from the same kernels on a
    quiet GPU: after the timed region one context maps --iso-batches batches back to
    back (every launch alone on the GPU, as `rocprofv3 --stats` of a --streams 1 run
    sees them), and the dominant kernel is the slot with the most device time there.
    The in-situ figure is kept as `in_situ`.  -> (roofline, quiet-GPU slots, fatal
    errors): a slot priced above the HBM peak (its alg. bytes are not the work it
    does) or a quiet-GPU dominant kernel longer than the step is an error."""
    pair_peak = VALU_INT32_OPS / OPS_PER_PAIR
    iso_prof, iso_cnt, iso_res, iso_nb = (quiet_gpu_profile(lib, L, devs[0], units, batches, P, opts, n_batches, args)
                                          if args.iso_batches > 0 else (None, None, None, 0))
    excluded = {}
    fatal = []
    if iso_prof:
        slots = {k: v for k, v in iso_prof.items() if v[1] > 0}
        # the figure called frac must fit the step (its kernel time per step <= ms_per_step).  A
        # tail-bound kernel (C5's k_chain_long: one wave on its longest segment for most of the
        # launch) can take longer on the quiet GPU than the whole step, where the other contexts'
        # kernels fill its idle CUs; such a slot is named in `excluded` and the next one is used
        def fits(k):
            return slots[k][0] / max(iso_nb, 1) <= ms_per_step * 1.0001
        for k in sorted(slots, key=lambda k: -slots[k][0]):
            if fits(k):
                break
            excluded[k] = {"quiet_ms_per_step": round(slots[k][0] / max(iso_nb, 1), 4),
                           "reason": "quiet-GPU time per step exceeds the in-situ step (tail-bound; contexts overlap it)"}
        dom = max((k for k in slots if k not in excluded), key=lambda k: slots[k][0], default=max(slots, key=lambda k: slots[k][0]))
        d_ms, d_calls = slots[dom]
        d_bytes = alg_bytes(iso_cnt, iso_res).get(dom, 0)
        frac_src = f"quiet GPU: one context, {iso_nb} batches x {P} units mapped back to back after the timed region"
        launches_per_step = d_calls / max(iso_nb, 1)
        share = d_ms / max(sum(v[0] for v in slots.values()), 1e-9)
    else:   # --iso-batches 0: the in-situ figure (its launches overlap other contexts' kernels)
        slots = timed_slots
        dom = max(slots, key=lambda k: slots[k][0])
        d_ms, d_calls = slots[dom]
        d_bytes = kb.get(dom, 0)
        frac_src = "in situ (--iso-batches 0)"
        launches_per_step = d_calls / max(args.steps, 1)
        share = d_ms / max(sum(v[0] for v in slots.values()), 1e-9)
    d_sym, d_hint = KERNEL_SYMBOLS.get(dom, (dom, ""))
    avg_s = d_ms / 1e3 / max(d_calls, 1)
    bytes_per_launch = d_bytes / max(d_calls, 1)
    achieved = bytes_per_launch / avg_s / 1e9 if avg_s > 0 else 0.0
    traffic, traffic_row = pmc_traffic(d_sym, d_hint, bench_config_tag(args))
    kernel_ms_per_step = avg_s * 1e3 * launches_per_step
    # the quiet-GPU figure called frac must fit the step (not the in-situ one, whose
    # launches include the other contexts' kernels)
    if iso_prof and kernel_ms_per_step > ms_per_step * 1.0001:
        fatal.append(f"roofline kernel {d_sym} takes {kernel_ms_per_step:.3f} ms per step "
                     f"({avg_s * 1e3:.4f} ms x {launches_per_step:g} launches) > the step's {ms_per_step:.3f} ms")
    ins = timed_slots.get(dom)
    in_situ = None
    if ins:
        ins_avg = ins[0] / 1e3 / ins[1]
        ins_ach = kb.get(dom, 0) / ins[1] / ins_avg / 1e9 if ins_avg > 0 else 0.0
        in_situ = {"avg_launch_ms": round(ins_avg * 1e3, 4), "launches_per_step": ins[1] / args.steps,
                   "achieved": round(ins_ach, 3), "frac": round(ins_ach / HBM_PEAK_GBS, 6),
                   "share_of_kernel_time": round(ins[0] / max(sum(v[0] for v in timed_slots.values()), 1e-9), 4),
                   "note": f"the timed region's launches ({max(1, args.streams)} contexts share the GPU: durations include "
                           f"the other contexts' kernels, so ms x launches may exceed the step)"}
    A_, Ar_, mk_, L_ = cnt["anchors"], cnt["rescued_anchors"], cnt["kept_minimizers"], cnt["bases"]
    B_path_ = (L_ + 3) // 4 + 16 * mk_ + 48 * A_ + 24 * Ar_
    path_frac = B_path_ / elapsed / 1e9 / HBM_PEAK_GBS if world == 1 else None
    roofline = {
        "bound": "hbm", "kernel": d_sym, "slot": dom, "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic, "traffic_row": traffic_row,
        "avg_launch_ms": round(avg_s * 1e3, 4), "launches_per_step": launches_per_step,
        "kernel_ms_per_step": round(kernel_ms_per_step, 4), "alg_bytes_per_launch": int(bytes_per_launch),
        "share_of_kernel_time": round(share, 4), "measured": frac_src, "excluded": excluded or None,
        "path_frac": round(path_frac, 6) if path_frac is not None else None,
        "path_note": "SURVEY.md §8d B(read) summed over the timed batches / step time / 8 TB/s (all kernels, host included)",
        "in_situ": in_situ,
        # SURVEY.md §8d secondary figure: DP pair evaluations against the int32 VALU rate at 15 ops per pair
        "compute": {"dp_pairs_per_step": cnt["dp_pairs"] / args.steps,
                    "pairs_per_s_wall": round(cnt["dp_pairs"] / elapsed, 1) if world == 1 else None,
                    "pairs_per_s_in_chain_kernels": round(cnt["dp_pairs"] / (chain_ms / 1e3), 1) if chain_ms > 0 else None,
                    "peak_pairs_per_s": pair_peak,
                    "frac_wall": round(cnt["dp_pairs"] / elapsed / pair_peak, 6) if world == 1 else None,
                    "note": "peak = 7.9e13 int32 ops/s / 15 ops per pair (SURVEY.md §8d); chain-kernel time overlaps "
                            "other contexts' kernels, so the in-kernel rate is a lower bound"},
        "seed_lookup_floor_bytes_per_step": 128 * cnt["kept_minimizers"] // args.steps,
        "seed_lookup_note": "a hashed-table probe reads at least one 128-B request per kept minimizer "
                            "(MI355X_MICROARCH.md: 128-B requests), against 16 B of table entry priced as algorithmic",
    }
    iso = None
    if iso_prof:   # every slot on the quiet GPU (ms per batch, launches, alg GB/s)
        ib = alg_bytes(iso_cnt, iso_res)
        iso = {"batches": iso_nb, "per_kernel": {
            k: {"ms_per_batch": round(v[0] / iso_nb, 4), "launches_per_batch": v[1] / iso_nb,
                "alg_GBps": round(ib.get(k, 0) / (v[0] / 1e3) / 1e9, 2) if v[0] > 0 else None}
            for k, v in sorted(iso_prof.items(), key=lambda kv: -kv[1][0]) if v[1] > 0},
            "kernel_ms_per_batch": round(sum(v[0] for v in iso_prof.values()) / iso_nb, 4)}
    # a slot above the HBM peak is not doing the work it is priced at
    over = [f"{k} {e['alg_GBps']} GB/s in situ" for k, e in per_kernel.items() if (e.get("alg_GBps") or 0) > HBM_PEAK_GBS]
    if iso:
        over += [f"{k} {e['alg_GBps']} GB/s quiet" for k, e in iso["per_kernel"].items() if (e.get("alg_GBps") or 0) > HBM_PEAK_GBS]
    if over:
        fatal.append("algorithmic bytes priced above the 8 TB/s HBM peak: " + ", ".join(over))
    return roofline, iso, fatal


def quiet_gpu_profile(lib, L, d0, units, batches, P, opts, n_batches, args):
    """Rank 0, after the timed region: one context maps the first --iso-batches
    batches' units back to back with per-kernel HIP events on (nothing else on
    the GPU).  -> (prof {slot: (ms, calls)}, summed counters, results, batches)."""
    nb = max(1, min(args.iso_batches, n_batches))
    d0.prof_reset()
    d0.prof_enable(True)
    cnt_i, res_i = {}, []
    for u in units[:nb * P]:
        rb = batches[u["b"]][0]
        L.check(lib.mm2g_batch_set_reads(d0._h, rb.ctypes.data_as(C.c_void_p), u["offs"].ctypes.data_as(L._P64), u["n"]), "set_reads")
        L.check(lib.mm2g_batch_map(d0._h, C.byref(opts)), "batch_map")
        L.check(lib.mm2g_batch_results(d0._h, u["res"], u["n"]), "batch_results")
        for k, v in d0.counters().items():
            cnt_i[k] = cnt_i.get(k, 0) + v
        res_i.append(np.frombuffer(u["res"], dtype=RES_DTYPE, count=u["n"]).copy())
    pi = d0.prof()
    d0.prof_enable(False)
    return pi, cnt_i, np.concatenate(res_i), nb


def read_name(rank: int, b: int, i: int) -> str:
    """Read i of batch b on this rank: names are unique over the ranks, since the
    parity check gathers every rank's sample into one PAF keyed by name."""
    return f"r{b}_{i}" if rank == 0 else f"r{b}_{i}_rank{rank}"


def sample_reads(args, batches, timed, n_sample: int, S: int, rank: int = 0):
    """The first reads of every timed batch (spread over all of them), with the
    GPU's per-read results and PAF lines: what the oracle re-checks."""
    if n_sample <= 0:
        return None
    by_batch = {}
    for u in timed:
        by_batch.setdefault(u["b"], []).append(u)
    bs = sorted(by_batch)
    per = max(1, -(-n_sample // len(bs)))
    out = {"reads": [], "res": [], "paf": {}}
    for b in bs:
        rb, offs = batches[b]
        us = sorted(by_batch[b], key=lambda u: u["k"])
        lines = {}
        for u in us:
            lines.update(paf_lines_by_read(bytes(u["buf"].raw[:u["len"]])))
        res = np.concatenate([np.frombuffer(u["res"], dtype=RES_DTYPE, count=u["n"]) for u in us if u["n"]])
        for i in range(min(per, len(offs) - 1)):
            nm = read_name(rank, b, i)
            out["reads"].append((nm, bytes(rb[int(offs[i]):int(offs[i + 1])])))
            out["res"].append(res[i].tobytes())
            if nm in lines:
                out["paf"][nm] = lines[nm]
    return out


REC_CMP = ("flags", "n_anchors", "score", "cm", "qs", "qe", "ts", "te", "rid", "rev")


def oracle_check(args, names, lens, gbuf, mid, thr, gathered, world):
    """Rank 0: the oracle (oracle/, C++ restatement of the reference align) on
    every rank's sample: PAF lines and per-read outcomes (incl. Q19 panic
    reads) vs the GPU's; and, at N=1, the CPU baseline (1 thread and all
    cores, median of 3) on that sample."""
    from oracle import oracle as O
    import tempfile

    O.set_quiet(True)
    t0 = time.time()
    oi = O.OIndex.build_from_buffer(names, gbuf, lens, w=10, k=15, b=14, flag=0, threads=thr)
    log(f"oracle index built in {time.time() - t0:.1f}s")
    reads = [r for s in gathered for r in s["reads"]]
    gpu_res = np.frombuffer(b"".join(r for s in gathered for r in s["res"]), dtype=RES_DTYPE)
    gpu_paf = {}
    for s in gathered:
        gpu_paf.update(s["paf"])
    seqs = [r[1] for r in reads]
    rnames = [r[0] for r in reads]
    rec = O.align_records(oi, seqs, mid_occ=mid, threads=thr, min_cnt=args.min_cnt)
    multi = args.min_cnt <= 1 and args.min_chain_score <= 15
    copt = {"min_cnt": args.min_cnt, "min_chain_score": args.min_chain_score}
    diff = []
    # (per-read records follow the reference's -m 40 best chain; under a non-default -m the PAF lines are the check)
    for i in range(len(seqs) if args.min_chain_score == 40 else 0):
        g = tuple(int(gpu_res[f][i]) for f in REC_CMP)
        g = (g[0] & 11,) + g[1:]
        w = tuple(int(v) for v in rec[i][:10])
        if g != w:
            diff.append(rnames[i])
    cat = np.frombuffer(b"".join(seqs), dtype=np.uint8)
    offs = np.zeros(len(seqs) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(x) for x in seqs])
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "cpu.paf")
        oi.align_buffer(rnames, cat, offs, out, mid_occ=mid, threads=thr, **copt)
        cpu_lines = paf_lines_by_read(open(out, "rb").read())
    paf_same = cpu_lines == gpu_paf
    # paf.rs:178's binary_search as rustc 1.52-1.81 compiles it (the device and the
    # oracle default follow >= 1.82): how many sampled reads would change
    O.set_binary_search(True)
    try:
        with tempfile.TemporaryDirectory() as td:
            out = os.path.join(td, "cpu_pre182.paf")
            oi.align_buffer(rnames, cat, offs, out, mid_occ=mid, threads=thr, **copt)
            pre_lines = paf_lines_by_read(open(out, "rb").read())
    finally:
        O.set_binary_search(False)
    bs_diff = sum(1 for k in set(cpu_lines) | set(pre_lines) if cpu_lines.get(k) != pre_lines.get(k))
    panics = int(((rec[:, 0] & 8) != 0).sum())
    parity = {"reads": len(seqs), "ranks_sampled": world, "identical": bool(paf_same and not diff),
              "paf_lines_identical": bool(paf_same), "gpu_lines": len(gpu_paf), "cpu_lines": len(cpu_lines),
              "per_read_outcome_identical": not diff, "per_read_outcome_diffs": diff[:10],
              "cpu_panics": panics, "chain_opts": f"-n {args.min_cnt} -m {args.min_chain_score}" + (" (multi-chain output)" if multi else ""),
              "rustc_binary_search": {"assumed": ">= 1.82 (base/size halving)",
                                      "reads_whose_paf_differs_under_1_52_to_1_81": bs_diff,
                                      "note": "k = 15 is odd: minimizer positions are strictly increasing, so both std "
                                              "algorithms agree (DESIGN.md §2); tests/golden/binsearch_even_k.json pins both at k = 16"},
              "note": "per-read outcome = chain flags, anchors, score, cm, q/t ranges, rid, strand; it covers the reads "
                      "on which the reference panics (Q19), which have no PAF line on either side"}
    cpu = None
    if world == 1 and not args.no_cpu:
        # calibrate, then size the sample to ~cpu_seconds per run
        n_cal = min(20, len(seqs))
        _, _, t_cal = oi.align_buffer(rnames[:n_cal], cat, offs[:n_cal + 1], None, mid_occ=mid, threads=1, **copt)
        per_read = max(t_cal / max(n_cal, 1), 1e-4)
        n_s = int(min(len(seqs), max(n_cal, args.cpu_seconds / per_read)))
        bases = int(offs[n_s])
        t1 = [oi.align_buffer(rnames[:n_s], cat, offs[:n_s + 1], None, mid_occ=mid, threads=1, **copt)[2] for _ in range(3)]
        ncpu = affinity_cpus()   # every CPU in the affinity set, not the OMP_NUM_THREADS share
        tN = [oi.align_buffer(rnames[:n_s], cat, offs[:n_s + 1], None, mid_occ=mid, threads=ncpu, **copt)[2] for _ in range(3)]
        v1 = bases / statistics.median(t1) / 1e9
        vN = bases / statistics.median(tN) / 1e9
        pf = float(((rec[:n_s, 0] & 8) != 0).sum()) / max(n_s, 1)
        log(f"cpu baseline: {n_s} reads, 1 thread {t1} s, {ncpu} threads {tN} s")
        cpu = {"value": round(v1, 9), "unit": "Gbases/s", "cores": 1, "kind": "port",
               "sample": f"{n_s} reads ({bases / 1e6:.1f} Mb) spread over the timed steps' batches; oracle/ C++ restatement "
                         f"of mm2rs align (1 thread, as the reference), index build excluded, median of 3 runs; "
                         f"{pf * 100:.0f}% of these reads end in the reference's Q19 panic after the full per-read DP "
                         f"(their chaining cost is paid, only the PAF line is missing)",
               "runs_s": [round(x, 3) for x in t1],
               "cpu_model": cpu_model(), "nproc": os.cpu_count(),
               "all_cores": {"value": round(vN, 9), "cores": ncpu, "runs_s": [round(x, 3) for x in tN],
                             "note": f"{ncpu} threads, one per CPU in the process's affinity set ({os.cpu_count()} CPUs "
                                     f"on the host; OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')} is not "
                                     f"used for this leg); the same sample as the 1-thread leg"}}
    oi.close()
    return cpu, parity


if __name__ == "__main__":
    main()
