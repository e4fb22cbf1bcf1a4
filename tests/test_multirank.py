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
        t, b, every = bench.reduce_step_time(dist, elapsed=1.0 + rank, n_bases=1000 * (rank + 1), world=world, device="cpu")
        q.put((rank, t, b, bench.rank_read_seed(3, rank), every, bench.rank_times(every, 10)))
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
    assert [g[4] for g in got] == [[1.0, 2.0], [1.0, 2.0]]   # every rank's own time, in rank order
    rt = got[0][5]                                        # config fields of the bench line
    assert rt["per_rank_ms_per_step"] == [100.0, 200.0] and rt["rank_time_max_over_mean"] == round(200 / 150, 4)


def test_single_rank_no_collective():
    assert bench.reduce_step_time(None, 1.5, 42, 1, "cpu") == (1.5, 42.0, [1.5])
    assert bench.rank_times([1.5], 3) == {"per_rank_ms_per_step": [500.0], "rank_time_max_over_mean": 1.0}


def test_workload_reference_size_units():
    assert bench.ref_size(4_641_652) == "4.64 Mb" and bench.ref_size(3_088_269_832) == "3.09 Gb"


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


_RANK_SCRIPT = r'''
import os, sys, json
import torch, torch.distributed as dist
dist.init_process_group("gloo")
t = torch.ones(1)
dist.all_reduce(t)
out = {"rank": int(os.environ["RANK"]), "local": int(os.environ["LOCAL_RANK"]), "world": dist.get_world_size(),
       "seen": int(t.item()), "addr": os.environ["MASTER_ADDR"], "argv": sys.argv[1:],
       "spawned": os.environ.get("MM2G_BENCH_SPAWNED")}
with open(os.path.join(sys.argv[1], "rank%d.json" % out["rank"]), "w") as fh:
    json.dump(out, fh)
dist.destroy_process_group()
sys.exit(int(os.environ.get("FAIL_RANK", "-1")) == out["rank"] and 3 or 0)
'''


def test_self_spawn_starts_every_rank(tmp_path, monkeypatch):
    """`bench.py --gpus N` without a launcher starts N rank processes itself
    (here a stand-in rank script over gloo): every rank joins the collective
    and sees the launcher environment torch.distributed.run would give it."""
    import json
    import sys
    script = tmp_path / "rank.py"
    script.write_text(_RANK_SCRIPT)
    monkeypatch.delenv("FAIL_RANK", raising=False)
    rc = bench.spawn_ranks(3, [str(tmp_path), "--gpus", "3"], "gloo", 0, cmd=[sys.executable, str(script)])
    assert rc == 0
    got = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(3)]
    assert [g["rank"] for g in got] == [0, 1, 2] and [g["local"] for g in got] == [0, 1, 2]
    assert all(g["world"] == 3 and g["seen"] == 3 and g["addr"] == "127.0.0.1" and g["spawned"] == "1" for g in got)
    assert all(g["argv"] == [str(tmp_path), "--gpus", "3"] for g in got)


def test_self_spawn_failing_rank_fails_the_run(tmp_path, monkeypatch):
    import sys
    script = tmp_path / "rank.py"
    script.write_text(_RANK_SCRIPT)
    monkeypatch.setenv("FAIL_RANK", "1")
    rc = bench.spawn_ranks(2, [str(tmp_path)], "gloo", 0, cmd=[sys.executable, str(script)])
    assert rc == 3


def test_more_rccl_ranks_than_gpus_is_an_error():
    with pytest.raises(SystemExit) as e:
        bench.spawn_ranks(2, [], "nccl", 1)
    assert "2 GPUs" in str(e.value.code) or "needs 2" in str(e.value.code)


def test_rank_count_must_match_gpus():
    assert bench.rank_env(1, {}) == (0, 1, 0)
    assert bench.rank_env(4, {"WORLD_SIZE": "4", "RANK": "2", "LOCAL_RANK": "2"}) == (2, 4, 2)
    with pytest.raises(SystemExit):
        bench.rank_env(8, {})                     # --gpus 8 in one process: never a silent 1-GPU run
    with pytest.raises(SystemExit):
        bench.rank_env(2, {"WORLD_SIZE": "4", "RANK": "0"})


def _genome_worker(rank, world, port, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank), "WORLD_SIZE": str(world)})
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import hashlib
        args = bench.parse(["--preset", "ecoli", "--scale", "0.05"])
        names, lens, g = bench.shared_genome(args, dist, rank, world, 2, f"t{port}")
        q.put((rank, names, [int(x) for x in lens], hashlib.sha256(bytes(g)).hexdigest(), type(g).__name__))
    finally:
        dist.destroy_process_group()


def test_shared_genome_one_generator(tmp_path):
    """Rank 0 generates the reference once; the other ranks map it from /dev/shm
    and see the same bytes (the file is gone once every rank has it)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_genome_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got[0][1:4] == got[1][1:4] and sum(got[0][2]) > 0
    assert got[1][4] == "memmap"
    assert not os.path.exists(f"/dev/shm/mm2g_bench_t{port}.genome")


def _records_fastq(path, names, seqs):
    with open(path, "wb") as fh:
        for nm, s in zip(names, seqs):
            q = bytes(64 if i % 7 == 0 else 73 for i in range(len(s)))   # quality lines that start with '@'
            fh.write(b"@" + nm.encode() + b" extra\n" + s + b"\n+\n" + q + b"\n")


@pytest.mark.parametrize("fmt", ["fasta", "fastq"])
def test_read_range_partitions_records(tmp_path, fmt):
    """shard.read_range: the byte ranges of every world size hand each record
    to exactly one rank, in input order, parsed as SeqStream parses them
    (names to the first space, multi-line FASTA, FASTQ quality skipped)."""
    import random
    from minimap2_rs_amd.shard import read_range
    rng = random.Random(5)
    names = [f"q{i}" for i in range(37)]
    seqs = [bytes(rng.choice(b"ACGTN") for _ in range(rng.choice([0, 1, 50, 81, 160, 333]))) for _ in names]
    path = str(tmp_path / f"r.{fmt}")
    if fmt == "fasta":
        from tools import simdata
        simdata.write_fasta(path, names, seqs)
    else:
        _records_fastq(path, names, seqs)
    for world in (1, 2, 3, 5, 8, 40):
        got_n, got_s = [], []
        for r in range(world):
            nm, buf, offs = read_range(path, r, world)
            got_n += nm
            got_s += [bytes(buf[int(offs[i]):int(offs[i + 1])]) for i in range(len(nm))]
        assert got_n == names and got_s == seqs, world
    empty = str(tmp_path / "empty.fa")
    open(empty, "wb").close()
    nm, buf, offs = read_range(empty, 0, 2)
    assert nm == [] and len(offs) == 1


def test_read_names_unique_over_ranks():
    """bench.py's parity check gathers every rank's sampled PAF into one dict keyed by read name."""
    names = {bench.read_name(r, b, i) for r in range(8) for b in range(3) for i in range(50)}
    assert len(names) == 8 * 3 * 50 and bench.read_name(0, 2, 7) == "r2_7"
