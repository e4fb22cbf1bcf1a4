"""CPU: bench.py's algorithmic-byte pricing follows the work to
the kernel that does it -- the sort slots by the class the library dispatched
each read to (counters 18-20), fused seeding charged to the sort that seeds
(counters 16/17 for k_sort_read, 21/22 for k_sort_big) and taken off
k_seed_write -- so a slot is never priced for work another kernel did."""
import numpy as np

import bench
from minimap2_rs_amd import api


def _res(n_anchors):
    r = np.zeros(len(n_anchors), dtype=bench.RES_DTYPE)
    r["n_anchors"] = n_anchors
    r["flags"] = 1
    return r


def _cnt(**kw):
    c = {k: 0 for k in ("bases", "minimizers", "kept_minimizers", "anchors", "rescued_anchors", "dp_pairs", "dp_anchors")}
    c.update(kw)
    return c


def test_counter_names_cover_the_abi():
    """api.Device.counters() names every MM2G_N_COUNTERS slot (include/mm2g.h)."""
    import re
    import inspect
    hdr = open(bench.os.path.join(bench.ROOT, "include", "mm2g.h")).read()
    n = int(re.search(r"#define MM2G_N_COUNTERS (\d+)", hdr).group(1))
    src = inspect.getsource(api.Device.counters)
    keys = re.findall(r'"([a-z_0-9]+)"', src.split("buf =")[0])
    assert len(keys) == n and len(set(keys)) == n, (n, keys)
    for k in ("sort_small_anchors", "sort_cell_anchors", "sort_whole_anchors", "fused_big_anchors", "fused_big_minimizers"):
        assert k in keys


def test_sort_classes_from_counters():
    # multi-chain output (no singleton filter): the large reads go whole to k_sort_radix
    res = _res([3000, 20000, 20000])
    cnt = _cnt(anchors=43000, minimizers=4000, sort_small_anchors=3000, sort_cell_anchors=0, sort_whole_anchors=40000)
    b = bench.alg_bytes(cnt, res)
    assert b["sort_small"] == 16 * 3000 and b["sort_large"] == 0 and b["sort_radix"] == 16 * 40000
    # the same reads with the filter on: the cell path takes them (thresholds never consulted)
    cnt.update(sort_cell_anchors=40000, sort_whole_anchors=0)
    b = bench.alg_bytes(cnt, res)
    assert b["sort_large"] == 16 * 40000 and b["sort_radix"] == 0


def test_fused_seeding_priced_where_it_runs():
    res = _res([20000, 200000])
    cnt = _cnt(anchors=220000, minimizers=20000, sort_cell_anchors=20000, sort_whole_anchors=200000,
               fused_anchors=20000, fused_minimizers=1800, fused_big_anchors=200000, fused_big_minimizers=18000)
    b = bench.alg_bytes(cnt, res)
    assert b["seed_write"] == 12 * (20000 - 1800 - 18000)          # no anchor left for k_seed_write
    assert b["sort_large"] == 16 * 20000 + 12 * 1800 + 8 * 20000
    assert b["sort_big"] == 16 * 200000 + 12 * 18000 + 8 * 200000
    # nothing fused: k_seed_write writes every key
    cnt.update(fused_anchors=0, fused_minimizers=0, fused_big_anchors=0, fused_big_minimizers=0)
    b = bench.alg_bytes(cnt, res)
    assert b["seed_write"] == 12 * 20000 + 16 * 220000 and b["sort_big"] == 16 * 200000


def test_old_counter_sets_fall_back_to_thresholds():
    """Counter dicts without 18-20 (older libraries) price by the read-size thresholds."""
    res = _res([1, 100, bench.SORT_SMALL + 1, bench.SORT_CELL_MAX + 1])
    b = bench.alg_bytes(_cnt(anchors=int(res["n_anchors"].sum())), res)
    assert b["sort_small"] == 16 * 100
    assert b["sort_large"] == 16 * (bench.SORT_SMALL + 1)
    assert b["sort_big"] == 16 * (bench.SORT_CELL_MAX + 1)
