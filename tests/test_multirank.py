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
