"""CPU, world_size 2 over gloo: the multi-GPU bench logic (one process per
GPU, reads sharded by rank with no data-path collective, barrier +
max-over-ranks time, whole-job bases) exercised on the CPU."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from minimap2_rs_amd.shard import gather_paf, shard_cuts


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank), "WORLD_SIZE": str(world)})
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dist.barrier()
        t, b = bench.reduce_step_time(dist, elapsed=1.0 + rank, n_bases=1000 * (rank + 1), world=world, device="cpu")
        q.put((rank, t, b, bench.rank_read_seed(3, rank)))
    finally:
        dist.destroy_process_group()


def test_reduce_over_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    got = sorted(q.get(timeout=5) for _ in range(2))
    assert [g[1] for g in got] == [2.0, 2.0]              # max over ranks
    assert [g[2] for g in got] == [3000.0, 3000.0]        # whole-job bases
    assert got[0][3] != got[1][3]                         # each rank maps its own reads


def test_single_rank_no_collective():
    assert bench.reduce_step_time(None, 1.5, 42, 1, "cpu") == (1.5, 42.0)


@pytest.mark.parametrize("n,s", [(10000, 1), (10000, 3), (7, 3), (0, 2), (5, 8)])
def test_share_cuts(n, s):
    c = bench.share_cuts(n, s)
    assert c[0] == 0 and c[-1] == n and len(c) == max(1, s) + 1
    assert all(a <= b for a, b in zip(c, c[1:]))


def _shard_worker(rank, world, port, ref, reads_fa, q):
    """One rank: its contiguous shard of the reads (balanced by bases), mapped
    on its own (the CPU oracle stands in for the device here: no GPU on this
    box), PAF gathered to rank 0 in rank order."""
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank), "WORLD_SIZE": str(world)})
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import tempfile
        import numpy as np
        from oracle import oracle as O
        recs = O.read_fasta(reads_fa)
        cuts = shard_cuts([len(s) for _, s in recs], world)
        mine = recs[cuts[rank]:cuts[rank + 1]]
        oi = O.OIndex.build(ref, 10, 15, 14, 0, 2)
        with tempfile.TemporaryDirectory() as td:
            out = os.path.join(td, "p.paf")
            cat = np.frombuffer(b"".join(s for _, s in mine) or b"\0", np.uint8)
            offs = np.zeros(len(mine) + 1, np.uint64)
            offs[1:] = np.cumsum([len(s) for _, s in mine])
            oi.align_buffer([n for n, _ in mine], cat, offs, out, threads=1)
            paf = open(out, "rb").read()
        allp = gather_paf(dist, paf, rank, world)
        q.put((rank, cuts, len(mine), allp))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_map_gathers_in_input_order(tmp_path, world):
    """Reads sharded over `world` gloo ranks by shard_cuts, PAF gathered to rank
    0: byte-identical to one process mapping every read."""
    from oracle import oracle as O
    from tools import simdata
    ref = str(tmp_path / "ref.fa")
    reads = str(tmp_path / "reads.fa")
    simdata.write_genome("small", 1.0, 11, ref)
    simdata.write_reads(ref, 60, 3000, 12, reads)
    want_p = str(tmp_path / "want.paf")
    O.OIndex.build(ref, 10, 15, 14, 0, 2).align_fasta(reads, want_p)
    want = open(want_p, "rb").read()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_shard_worker, args=(r, world, port, ref, reads, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert sum(g[2] for g in got) == 60 and all(g[2] > 0 for g in got)
    assert got[0][3] == want and want.count(b"\n") > 20
    assert all(g[3] == b"" for g in got[1:])


@pytest.mark.parametrize("lens,world", [([10] * 10, 2), ([100, 1, 1, 1, 1], 2), ([5, 5, 5], 5), ([], 3), ([7], 1)])
def test_shard_cuts_balanced(lens, world):
    c = shard_cuts(lens, world)
    assert len(c) == world + 1 and c[0] == 0 and c[-1] == len(lens)
    assert all(a <= b for a, b in zip(c, c[1:]))
    if lens and world <= len(lens):
        tot = sum(lens)
        part = [sum(lens[c[r]:c[r + 1]]) for r in range(world)]
        assert max(part) <= tot / world + max(lens)


def test_batches_distinct_per_rank_and_step():
    seeds = {bench.batch_seed(3, r, b) for r in range(8) for b in range(40)}
    assert len(seeds) == 8 * 40 and bench.batch_seed(3, 0, 0) == 3
