"""Read sharding over GPUs (BASELINE config C4): one process per
GPU, contiguous read ranges, the index replicated on every GPU, no collective
on the data path, PAF gathered to rank 0 in input order afterwards (the
reference maps reads independently, Q10, and prints them in input order,
src/main.rs:189-230, so the concatenation equals a single-process run).

As a program (the multi-process form of ``mm2rs align``)::

    python -m minimap2_rs_amd.shard <ref.mmi|ref.fa> <reads.fa|fq> -o out.paf --gpus N
    python -m torch.distributed.run --nproc-per-node N -m minimap2_rs_amd.shard ... --gpus N

Rank r maps the records whose header starts in the r-th of N equal byte ranges
of the read file (balanced by bytes ~ bases; each rank reads only its own
range), on GPU ``LOCAL_RANK`` through libmm2g.so with ``--streams`` contexts
sharing one device index.  A FASTA reference is indexed once, on rank 0's GPU,
and handed to the other ranks as a .mmi in /dev/shm (mapped, bucket-parallel
load).  ``MM2G_DIST_BACKEND=gloo`` rehearses N ranks on fewer GPUs (ranks share
a device); with RCCL (the default) more ranks than GPUs is an error.

``shard_cuts`` / ``gather_paf`` are also used by callers holding the reads in
memory (tests/test_multirank.py); bench.py's weak-scaling run gives every rank
its own reads instead.
"""
from __future__ import annotations

import argparse
import json
import mmap
import os
import socket
import subprocess
import sys
import threading
import time
from typing import List, Sequence, Tuple

import numpy as np


def shard_cuts(lens: Sequence[int], world: int) -> List[int]:
    """Contiguous read ranges [cuts[r], cuts[r+1]) for `world` ranks with
    about equal numbers of bases each (reads are never split)."""
    world = max(1, int(world))
    n = len(lens)
    if n == 0:
        return [0] * (world + 1)
    c = np.concatenate([[0], np.cumsum(np.asarray(lens, dtype=np.int64))])
    total = int(c[-1])
    cuts = [0]
    for r in range(1, world):
        # first read whose start reaches r/world of the bases
        cuts.append(max(cuts[-1], int(np.searchsorted(c, total * r / world, side="left"))))
    cuts.append(n)
    return [min(x, n) for x in cuts]


def gather_paf(dist, paf: bytes, rank: int, world: int) -> bytes:
    """All ranks' PAF text concatenated in rank order (= input order for
    shard_cuts ranges) on rank 0; b"" elsewhere.  Outside any timed region."""
    if world <= 1:
        return paf
    got = [None] * world if rank == 0 else None
    dist.gather_object(paf, got, dst=0)
    return b"".join(got) if rank == 0 else b""


# ---- byte-range sharding of a FASTA / FASTQ file -----------------------------

def _is_fastq(mm) -> bool:
    for i in range(len(mm)):
        c = mm[i:i + 1]
        if c in (b">", b"@"):
            return c == b"@"
    return False


def _line_start(mm, p: int) -> int:
    """First line start at or after p."""
    if p <= 0:
        return 0
    if mm[p - 1:p] == b"\n":
        return p
    q = mm.find(b"\n", p)
    return len(mm) if q < 0 else q + 1


def record_start(mm, p: int, fastq: bool) -> int:
    """The first record start at or after byte p (len(mm) if none): a line
    starting with '>' (FASTA), or '@' with its second next line starting with
    '+' (4-line FASTQ: a quality line may start with '@', but the line two after
    it is a sequence line).  Every rank applies the same rule, so rank r's end
    is rank r+1's start and each record lands on exactly one rank."""
    n = len(mm)
    p = _line_start(mm, p)
    while p < n:
        c = mm[p:p + 1]
        if not fastq and c == b">":
            return p
        if fastq and c == b"@":
            l1 = _line_start(mm, p + 1)
            l2 = _line_start(mm, l1 + 1) if l1 < n else n
            if l2 < n and mm[l2:l2 + 1] == b"+":
                return p
        q = mm.find(b"\n", p)
        if q < 0:
            return n
        p = q + 1
    return n


def read_range(path: str, rank: int, world: int) -> Tuple[List[str], np.ndarray, np.ndarray]:
    """The records whose first byte lies in the rank-th of `world` equal byte
    ranges of `path`, parsed as the library's SeqStream parses them (name =
    header text up to the first space or tab; FASTA sequence lines
    concatenated; FASTQ quality skipped).  -> (names, bases, offsets)."""
    with open(path, "rb") as fh:
        size = os.fstat(fh.fileno()).st_size
        if size == 0:
            return [], np.zeros(1, np.uint8), np.zeros(1, np.uint64)
        with mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ) as mm:
            fastq = _is_fastq(mm)
            lo = record_start(mm, size * rank // world, fastq) if rank else record_start(mm, 0, fastq)
            hi = record_start(mm, size * (rank + 1) // world, fastq) if rank + 1 < world else size
            lines = mm[lo:hi].split(b"\n")
    names, parts, lens = [], [], []
    i = 0
    while i < len(lines):
        ln = lines[i].rstrip(b"\r")
        i += 1
        if not ln or ln[:1] not in (b">", b"@"):
            continue
        name = ln[1:].split(b" ", 1)[0].split(b"\t", 1)[0].decode()
        seq = []
        if ln[:1] == b"@":
            while i < len(lines):
                s = lines[i].rstrip(b"\r")
                i += 1
                if s[:1] == b"+":
                    break
                seq.append(s)
            need, got = sum(len(s) for s in seq), 0
            while got < need and i < len(lines):
                got += len(lines[i].rstrip(b"\r"))
                i += 1
        else:
            while i < len(lines) and lines[i][:1] != b">":
                seq.append(lines[i].rstrip(b"\r"))
                i += 1
        s = b"".join(seq)
        names.append(name)
        parts.append(s)
        lens.append(len(s))
    buf = np.frombuffer(b"".join(parts), dtype=np.uint8) if sum(lens) else np.zeros(1, np.uint8)
    offs = np.zeros(len(lens) + 1, np.uint64)
    offs[1:] = np.cumsum(np.asarray(lens, dtype=np.uint64))
    return names, buf, offs


# ---- launching --------------------------------------------------------------

def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n: int, cmd: Sequence[str], log=print) -> int:
    """Start the n rank processes of `cmd` as fresh children with the
    environment torch.distributed.run gives them, and wait (the caller never
    touches a GPU, so nothing is exec'd from a GPU process).  One failing rank
    stops the others; the exit code is the first failure's."""
    port = free_port()
    base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n), MM2G_BENCH_SPAWNED="1")
    procs = [subprocess.Popen(list(cmd), env=dict(base, RANK=str(r), LOCAL_RANK=str(r))) for r in range(n)]
    log(f"started {n} rank processes (pids {[p.pid for p in procs]}, master 127.0.0.1:{port})")
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            c = p.poll()
            if c is None:
                continue
            alive.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                log(f"rank process {p.pid} exited with {c}; stopping the others")
                for q in alive:
                    q.terminate()
        time.sleep(0.1)
    return rc


# ---- one rank ---------------------------------------------------------------

def map_records(devs, names: Sequence[str], buf: np.ndarray, offs: np.ndarray, opts, batch_reads: int) -> bytes:
    """PAF of the records, in order: batches of `batch_reads` pulled by the
    contexts (one host thread each, so one batch's packing and PAF formatting
    overlap another's device work)."""
    from . import api
    n = len(names)
    cuts = list(range(0, n, max(1, batch_reads))) + [n]
    jobs = list(zip(cuts[:-1], cuts[1:]))
    out = [b""] * len(jobs)
    nxt, lock, errs = [0], threading.Lock(), []

    def worker(d: "api.Device"):
        try:
            while True:
                with lock:
                    j = nxt[0]
                    nxt[0] += 1
                if j >= len(jobs):
                    return
                lo, hi = jobs[j]
                d.set_reads_packed(buf, offs[lo:hi + 1])
                d.map(opts)
                out[j] = d.batch_paf(list(names[lo:hi])).encode()
        except Exception as e:   # surfaced after the join
            errs.append(e)
    ths = [threading.Thread(target=worker, args=(d,)) for d in devs]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    if errs:
        raise errs[0]
    return b"".join(out)


def _log(*a):
    print("[shard]", *a, file=sys.stderr, flush=True)


def parse(argv=None):
    p = argparse.ArgumentParser(prog="python -m minimap2_rs_amd.shard",
                                description="mm2rs align with reads sharded over one process per GPU (SURVEY.md §8e)")
    p.add_argument("target", help="reference .mmi or FASTA")
    p.add_argument("query", help="reads, FASTA or 4-line FASTQ")
    p.add_argument("-o", "--out", default="-", help="PAF output (rank 0; '-' = stdout)")
    p.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); without a launcher they are self-spawned")
    p.add_argument("-w", type=int, default=10)
    p.add_argument("-k", type=int, default=15)
    p.add_argument("-b", type=int, default=14)
    p.add_argument("-H", dest="hpc", action="store_true")
    p.add_argument("-f", type=float, default=2e-4, help="mid_occ fraction (main.rs:196-197)")
    p.add_argument("-g", type=int, default=None, help="max gap")
    p.add_argument("-r", default=None, help="bw[,bw_long]")
    p.add_argument("-n", type=int, default=None)
    p.add_argument("-m", type=int, default=None)
    p.add_argument("-t", "--threads", type=int, default=16, help="host threads for the index build / .mmi load")
    p.add_argument("--streams", type=int, default=2, help="contexts per GPU")
    p.add_argument("--batch-reads", type=int, default=5000)
    p.add_argument("--report", default=None, help="rank 0 writes a JSON summary of the run here")
    return p.parse_args(argv)


def _opts(args):
    from . import api
    kw = {"w": args.w, "k": args.k}
    if args.g is not None:
        kw["max_gap"] = args.g
    if args.r is not None:
        bw = args.r.split(",")
        kw["bw"] = int(bw[0])
        if len(bw) > 1:
            kw["bw_long"] = int(bw[1])
    if args.n is not None:
        kw["min_cnt"] = args.n
    if args.m is not None:
        kw["min_chain_score"] = args.m
    return api.map_opts(**kw)


def _index(args, dist, rank: int, world: int, gpu: int):
    """The host index on every rank: a .mmi is mapped by each rank; a FASTA is
    built once on rank 0's GPU and handed over as a .mmi in /dev/shm (each rank
    builds its own when /dev/shm has no room)."""
    from . import api
    flag = 1 if args.hpc else 0
    if args.target.endswith(".mmi"):
        return api.Index.load_from_mmi(args.target)

    def build():
        return api.Index.build_index_from_fasta_gpu(args.target, args.w, args.k, args.b, flag, gpu, args.threads)
    if world <= 1:
        return build()
    shm = f"/dev/shm/mm2g_shard_{os.environ.get('MASTER_PORT', '0')}.mmi"
    idx, ok = None, [False]
    if rank == 0:
        idx = build()
        try:
            idx.save_to_mmi(shm)
            ok = [True]
        except Exception as e:
            _log(f"rank 0: .mmi to {shm} failed ({e}); every rank builds its own index")
    dist.broadcast_object_list(ok, src=0)
    if rank != 0:
        idx = api.Index.load_from_mmi(shm) if ok[0] else build()
    dist.barrier()
    if rank == 0 and ok[0]:
        os.unlink(shm)
    return idx


def main(argv=None) -> int:
    args = parse(argv)
    backend = os.environ.get("MM2G_DIST_BACKEND", "nccl")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        import torch
        ndev = torch.cuda.device_count()      # counts devices without initialising HIP on this image
        if backend == "nccl" and ndev < args.gpus:
            raise SystemExit(f"shard: --gpus {args.gpus} needs {args.gpus} GPUs for RCCL ranks, {ndev} visible "
                             f"(MM2G_DIST_BACKEND=gloo rehearses more ranks than GPUs)")
        return spawn_ranks(args.gpus, [sys.executable, "-m", "minimap2_rs_amd.shard"] + list(sys.argv[1:] if argv is None else argv),
                           log=_log)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world != args.gpus:
        raise SystemExit(f"shard: --gpus {args.gpus} but WORLD_SIZE={world}")
    import torch
    import torch.distributed as dist
    ndev = torch.cuda.device_count()
    if backend == "nccl" and world > max(ndev, 1):
        raise SystemExit(f"shard: {world} RCCL ranks but {ndev} GPU(s) visible")
    gpu = local % max(ndev, 1)
    seen = 1
    if world > 1:
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
        one = torch.ones(1, dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(one)
        seen = int(one.item())
        if seen != world:
            raise SystemExit(f"shard: all-reduce saw {seen} ranks, expected {world}")
    from . import api
    if api.load().mm2g_device_count() <= 0:
        raise SystemExit("shard: no HIP device visible")
    t0 = time.time()
    idx = _index(args, dist, rank, world, gpu)
    devs = [api.Device(gpu) for _ in range(max(1, args.streams))]
    devs[0].upload_index(idx, 10)
    mid = max(devs[0].index_mid_occ(args.f), 10)          # main.rs:196-197, from the device table's histogram
    devs[0].set_mid_occ(mid)
    for d in devs[1:]:
        d.share_index(devs[0], mid)
    idx.release_tables()
    t_index = time.time() - t0
    t0 = time.time()
    names, buf, offs = read_range(args.query, rank, world)
    t_read = time.time() - t0
    t0 = time.time()
    paf = map_records(devs, names, buf, offs, _opts(args), args.batch_reads)
    t_map = time.time() - t0
    mine = {"rank": rank, "gpu": gpu, "reads": len(names), "bases": int(offs[-1]), "index_s": round(t_index, 3),
            "read_s": round(t_read, 3), "map_s": round(t_map, 3), "paf_lines": paf.count(b"\n")}
    every = [mine]
    if world > 1:
        every = [None] * world
        dist.all_gather_object(every, mine)
    allp = gather_paf(dist, paf, rank, world)
    if rank == 0:
        if args.out == "-":
            sys.stdout.buffer.write(allp)
            sys.stdout.flush()
        else:
            with open(args.out, "wb") as fh:
                fh.write(allp)
        rep = {"ranks": world, "collective_backend": dist.get_backend() if world > 1 else None,
               "collective_world_seen": seen, "mid_occ": mid, "per_rank": every,
               "reads": sum(e["reads"] for e in every), "bases": sum(e["bases"] for e in every),
               "gbases_per_s_map": round(sum(e["bases"] for e in every) / max(max(e["map_s"] for e in every), 1e-9) / 1e9, 6)}
        _log(json.dumps(rep))
        if args.report:
            with open(args.report, "w") as fh:
                json.dump(rep, fh)
    for d in devs:
        d.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
