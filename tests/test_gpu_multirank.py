"""GPU: configuration C4's sharded path with the HIP library on
every rank.  The box has one GPU, so the ranks share it over gloo
(MM2G_DIST_BACKEND=gloo); with RCCL each rank would own a GPU, and nothing
else in the path changes (one process per GPU, the index replicated, no
collective on the data path, PAF gathered in input order).

  - `python -m minimap2_rs_amd.shard` (the multi-process ``mm2rs align``):
    reads byte-range sharded over 2 and 3 rank processes, each mapping its
    shard through libmm2g.so; the PAF gathered on rank 0 is byte-identical to
    the oracle CLI's (FASTA and FASTQ input).
  - `bench.py --gpus 2` self-spawned on the full hg38-shaped index (rank 0
    builds it and hands it over as a .mmi in /dev/shm): both ranks join the
    collective, and both ranks' sampled reads equal the oracle's (PAF and
    per-read outcome, incl. Q19 panic reads).

The launching test process only counts devices: the ranks are fresh child
processes (never an exec from a process that initialised the GPU)."""
import json
import os
import subprocess
import sys

import pytest

from tools import simdata

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MM2RS_CPU = os.path.join(ROOT, "oracle", "build", "mm2rs-cpu")


def _env():
    return dict(os.environ, MM2G_DIST_BACKEND="gloo", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))


def _fastq(path, fa):
    names, seqs = simdata.read_fasta_seqs(fa)
    with open(path, "wb") as fh:
        for nm, s in zip(names, seqs):
            fh.write(b"@" + nm.encode() + b"\n" + s + b"\n+\n" + b"@" * len(s) + b"\n")


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,fmt", [(2, "fa"), (3, "fq")])
def test_shard_map_vs_oracle_cli(tmp_path, world, fmt):
    ref = str(tmp_path / "ref.fa")
    reads = str(tmp_path / "reads.fa")
    simdata.write_genome("hg38", 0.002, 41, ref)           # 24 contigs, ~6 Mb, hg38-shaped repeats
    simdata.write_reads(ref, 600, 5000, 42, reads)
    want = subprocess.run([MM2RS_CPU, "align", ref, reads], check=True, capture_output=True, timeout=300).stdout
    if fmt == "fq":        # the same records as FASTQ (the oracle CLI reads FASTA only)
        fq = str(tmp_path / "reads.fq")
        _fastq(fq, reads)
        reads = fq
    out, rep = str(tmp_path / "out.paf"), str(tmp_path / "rep.json")
    p = subprocess.run([sys.executable, "-m", "minimap2_rs_amd.shard", ref, reads, "-o", out, "--gpus", str(world),
                        "--batch-reads", "128", "--report", rep], cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=500)
    assert p.returncode == 0, p.stderr[-3000:]
    got = open(out, "rb").read()
    assert got == want and want.count(b"\n") > 300
    r = json.load(open(rep))
    assert r["ranks"] == world and r["collective_world_seen"] == world and r["collective_backend"] == "gloo"
    assert [e["rank"] for e in r["per_rank"]] == list(range(world))
    assert all(e["reads"] > 0 for e in r["per_rank"]) and r["reads"] == 600
    assert sum(e["paf_lines"] for e in r["per_rank"]) == want.count(b"\n")


@pytest.mark.timeout(900)
def test_bench_two_ranks_hg38(tmp_path):
    """bench.py --gpus 2 (the driver's multi-GPU line, self-spawned) on the
    full 3.09 Gb hg38-shaped index, 1,000 x 10 kb reads per rank per step."""
    p = subprocess.run([sys.executable, "-u", "bench.py", "--gpus", "2", "--reads", "1000", "--steps", "2", "--warmup", "1",
                        "--streams", "2", "--no-cpu"], cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=840)
    with open(tmp_path / "bench2.err", "w") as fh:
        fh.write(p.stderr)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    cfg = line["config"]
    assert cfg["ranks"] == 2 and cfg["collective_world_seen"] == 2 and cfg["collective_backend"] == "gloo"
    assert cfg["launch"] == "self-spawned ranks" and line["n_gpus"] == 1 and cfg["ref_bases"] > 3_000_000_000
    assert len(cfg["per_rank_ms_per_step"]) == 2 and line["value"] > 0
    par = line["extra"]["parity_vs_oracle"]
    assert par["ranks_sampled"] == 2 and par["reads"] == 1000
    assert par["identical"] and par["paf_lines_identical"] and par["per_read_outcome_identical"], par
    assert par["cpu_panics"] > 0 and par["gpu_lines"] > 100      # Q19 panic reads and printed lines both covered
    assert line["roofline"]["frac"] > 0
