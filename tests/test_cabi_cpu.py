"""C-ABI library and host logic on the CPU (no GPU calls).

* libsanta_hip.so loads and exports every entry point include/santa_hip.h
  declares, with the ctypes signatures of santa_hip._lib;
* the host-side generator is deterministic and produces valid Kaggle-shaped
  data; sh_ctx_create rejects invalid tables before touching a device;
* the sampler's host mirror: bijection, and the block geometry equals the
  reference's arithmetic (mpi_single.py:238-240, mpi_twins.py:244-246).
"""
import ctypes
import json
import os
import re

import numpy as np
import pytest

from conftest import ROOT
from santa_hip import _lib, data as D, sampler as S

HEADER = os.path.join(ROOT, "include", "santa_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*([a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("sh_ctx_create", "sh_solve_blocks", "sh_score", "sh_sample_blocks",
                 "lsap_solve_batched_i64", "lsap_solve_batched_f64", "sh_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    for name in declared_functions():
        assert hasattr(L, name), f"{name} declared in santa_hip.h but not exported"
    assert sorted(_lib.SIGNATURES) == declared_functions()
    assert L.sh_version() == 1


def test_synthetic_generator_deterministic_and_valid():
    a = D.synthetic(seed=9, nc=30000, ng=30, nq=1000, n_wish=12, n_good=400)
    b = D.synthetic(seed=9, nc=30000, ng=30, nq=1000, n_wish=12, n_good=400)
    assert np.array_equal(a.wish, b.wish) and np.array_equal(a.goodkids, b.goodkids)
    assert np.array_equal(a.types, b.types)
    c = D.synthetic(seed=10, nc=30000, ng=30, nq=1000, n_wish=12, n_good=400)
    assert not np.array_equal(a.wish, c.wish)
    # wishlists: distinct gift ids in range
    w = np.sort(a.wish, axis=1)
    assert (w[:, 1:] != w[:, :-1]).all() and w.min() >= 0 and w.max() < a.ng
    g = np.sort(a.goodkids, axis=1)
    assert (g[:, 1:] != g[:, :-1]).all() and g.min() >= 0 and g.max() < a.nc
    # baseline: every type used nq times, families share a gift
    assert (np.bincount(a.types, minlength=a.ng) == a.nq).all()
    tri, tw = a.families
    t = a.types
    assert (t[0:tri:3] == t[1:tri:3]).all() and (t[1:tri:3] == t[2:tri:3]).all()
    assert (t[tri:tri + tw:2] == t[tri + 1:tri + tw:2]).all()


def _ctx_create(wish, good, nc, ng, nq):
    h = ctypes.c_void_p()
    wish = np.ascontiguousarray(wish, dtype=np.int16)
    good = np.ascontiguousarray(good, dtype=np.int32)
    rc = _lib.lib().sh_ctx_create(ctypes.byref(h), 0, wish.ctypes.data_as(ctypes.c_void_p),
                                  wish.shape[1], good.ctypes.data_as(ctypes.c_void_p),
                                  good.shape[1], nc, ng, nq)
    return rc


def test_ctx_create_rejects_invalid_tables_without_gpu():
    sd = D.synthetic(seed=1, nc=20000, ng=20, nq=1000, n_wish=10, n_good=100)
    w = sd.wish.copy()
    w[5, 3] = w[5, 4]  # repeated gift in one wishlist
    assert _ctx_create(w, sd.goodkids, sd.nc, sd.ng, sd.nq) == _lib.SH_ERR_ARGS
    assert "repeated" in _lib.last_error()
    w = sd.wish.copy()
    w[0, 0] = sd.ng  # out of range
    assert _ctx_create(w, sd.goodkids, sd.nc, sd.ng, sd.nq) == _lib.SH_ERR_ARGS
    g = sd.goodkids.copy()
    g[2, 1] = g[2, 0]
    assert _ctx_create(sd.wish, g, sd.nc, sd.ng, sd.nq) == _lib.SH_ERR_ARGS
    assert _ctx_create(sd.wish, sd.goodkids, 0, sd.ng, sd.nq) == _lib.SH_ERR_ARGS


@pytest.mark.parametrize("n_wish", [10, 100])
def test_ctx_create_host_checks_pass_without_gpu(n_wish):
    """Valid tables pass every host-side check of sh_ctx_create -- including
    the C++ twins tile-entry decode against the float32 pair sums for every
    code pair -- and only the first device call fails here (no GPU): the
    error is SH_ERR_HIP, not SH_ERR_ARGS."""
    sd = D.synthetic(seed=1, nc=20000, ng=200, nq=100, n_wish=n_wish, n_good=100)
    rc = _ctx_create(sd.wish, sd.goodkids, sd.nc, sd.ng, sd.nq)
    assert rc == _lib.SH_ERR_HIP, (rc, _lib.last_error())


@pytest.mark.parametrize("count", [1, 2, 3, 17, 1000, 19968, 954880])
def test_feistel_is_a_bijection(count):
    f = S.Feistel(123, 4, count)
    p = f.perm(np.arange(count, dtype=np.uint64))
    assert p.min() >= 0 and p.max() < count
    assert np.unique(p).size == count


def test_block_geometry_matches_reference_arithmetic():
    tri, tw = S.family_sizes(1_000_000)
    assert (tri, tw) == (5001, 40000)
    # mpi_single.py:238-240 at its default block_size=2000 and at n=256
    for bs in (2000, 256):
        lo, count, nb = S.single_geometry(1_000_000, bs, tri, tw)
        assert nb == int((1_000_000 - 45001) / bs)
        rmd = 1000000 - 45001 - nb * bs
        assert (lo, lo + count) == (45001, 1_000_000 - rmd)
    assert S.single_geometry(1_000_000, 256, tri, tw)[2] == 3730
    # mpi_twins.py:244-246: block_size counts children (2 per pair)
    for pairs in (3000, 256):
        bs = 2 * pairs
        lo, count, nb = S.twin_geometry(tri, tw, pairs)
        assert nb == int(40000 / bs)
        twins_rmd = 40000 - nb * bs
        first = list(range(5001, 45001 - twins_rmd, 2))
        assert lo == first[0] and count == len(first) == nb * pairs
    assert S.twin_geometry(tri, tw, 256)[2] == 78


def test_sample_blocks_disjoint():
    rows = S.sample_blocks(5, 1, 45001, 954880, 1, 256, 3730)
    assert rows.shape == (3730, 256)
    assert np.unique(rows).size == rows.size
    assert rows.min() >= 45001 and rows.max() < 45001 + 954880
    tw = S.sample_blocks(5, 1, 5001, 19968, 2, 256, 78)
    assert ((tw - 5001) % 2 == 0).all() and np.unique(tw).size == tw.size


def test_slot_ids_match_pandas_groupby_rank():
    import pandas as pd
    rng = np.random.default_rng(0)
    types = rng.integers(0, 7, size=500).astype(np.int16)
    subm = pd.DataFrame({"ChildId": np.arange(500), "GiftId": types.astype(np.int64)})
    subm["gift_rank"] = subm.groupby("GiftId").rank() - 1          # mpi_single.py:224
    want = (subm["GiftId"] * 1000 + subm["gift_rank"]).astype(np.int64).values  # :225-226
    assert np.array_equal(D.slot_ids(types, 1000), want)


def test_submission_csv_roundtrip(tmp_path):
    t = np.array([3, 3, 1, 0, 2], dtype=np.int16)
    p = tmp_path / "sub.csv"
    D.write_submission(str(p), t)
    assert open(p).readline().strip() == "ChildId,GiftId"
    assert np.array_equal(D.read_submission(str(p)), t)


def test_v2_csv_readers(tmp_path):
    """child_wishlist_v2.csv / gift_goodkids_v2.csv: no header, column 0 the
    id, dropped as mpi_single.py:194,196 do with drop(0, 1)."""
    sd = D.synthetic(seed=3, nc=20000, ng=20, nq=1000, n_wish=10, n_good=100)
    wp, gp = tmp_path / "child_wishlist_v2.csv", tmp_path / "gift_goodkids_v2.csv"
    np.savetxt(wp, np.c_[np.arange(sd.nc), sd.wish], fmt="%d", delimiter=",")
    np.savetxt(gp, np.c_[np.arange(sd.ng), sd.goodkids], fmt="%d", delimiter=",")
    w, g = D.read_wishlist(str(wp)), D.read_goodkids(str(gp))
    assert w.dtype == np.int16 and g.dtype == np.int32
    assert np.array_equal(w, sd.wish) and np.array_equal(g, sd.goodkids)
    sub = tmp_path / "baseline_res.csv"
    D.write_submission(str(sub), sd.types)
    assert np.array_equal(D.read_submission(str(sub), sd.nc), sd.types)
    # a child without a gift is an error, not a silent -1
    open(sub, "w").write("ChildId,GiftId\n0,1\n2,1\n")
    with pytest.raises(ValueError):
        D.read_submission(str(sub), 3)


def test_hash_cost_host_mirror_shape():
    C = S.hash_matrix(7, 0, 16, 100)
    assert C.shape == (16, 16) and C.min() >= 0 and C.max() < 100
    assert np.array_equal(C, S.hash_matrix(7, 0, 16, 100))
    assert not np.array_equal(C, S.hash_matrix(7, 1, 16, 100))


def test_gift_types_outside_range_are_rejected_on_the_host(tmp_path):
    """Gift types index on-chip tables in the kernels: the host refuses a
    type outside [0, ng) (the reference's numpy indexing raises IndexError)
    before anything reaches the device."""
    from santa_hip.context import check_types
    check_types(np.array([0, 5, 9], dtype=np.int64), 10)
    for bad in ([0, 10, 3], [-1, 2, 3], [0, 1, 40000]):
        with pytest.raises(ValueError):
            check_types(np.array(bad, dtype=np.int64), 10)
    p = tmp_path / "sub.csv"
    open(p, "w").write("ChildId,GiftId\n0,1\n1,20\n2,3\n")
    assert np.array_equal(D.read_submission(str(p), 3), [1, 20, 3])
    with pytest.raises(ValueError):
        D.read_submission(str(p), 3, ng=20)
    open(p, "w").write("ChildId,GiftId\n0,1\n5,2\n")
    with pytest.raises(ValueError):
        D.read_submission(str(p), 3)


def test_lsap_front_end_routes_wide_integers_to_float64(monkeypatch):
    """linear_sum_assignment solves integers in int64 only while scipy's
    float64 arithmetic on them is exact; wider ranges and unsigned input
    with maximize=True take the float64 replay (no GPU call: the solver is
    stubbed and the dtype it receives is recorded)."""
    import torch
    from santa_hip import lsap
    seen = []

    def fake(C, with_cost=True, flags=0):
        seen.append(C.dtype)
        B, n, _ = C.shape
        return torch.arange(n, dtype=torch.int32).repeat(B, 1), None

    monkeypatch.setattr(lsap, "solve_batched", fake)
    monkeypatch.setattr(torch.Tensor, "to", lambda self, *a, **k: self)
    lsap.linear_sum_assignment(np.array([[1, 2], [3, 4]]), device="cpu")
    lsap.linear_sum_assignment(np.array([[1 << 50, 2], [3, 4]]), device="cpu")
    lsap.linear_sum_assignment(np.array([[1, 2], [3, 4]], dtype=np.uint8), maximize=True, device="cpu")
    lsap.linear_sum_assignment(np.array([[0.5, 2], [3, 4]]), device="cpu")
    assert seen == [torch.int64, torch.float64, torch.int64, torch.float64]


def test_bench_roofline_helpers():
    """bench.py's roofline plumbing on the CPU: the register-tile design's
    launch has up to two kernels (tile build + solve), and the stored HBM traffic
    comes only from a committed rocprofv3 summary of the same kernel source
    and launch size (otherwise null with a note naming the source hash); one
    kernel name that serves two launch sizes (the 4-wave kernel: the twins
    round and the 8-GPU shard) never borrows the other size's figures."""
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.design_kernels("santa_sp3_kernel (1-wave sparse register tile)") == \
        ["santa_tile_kernel", "santa_sp3_kernel"]
    assert bench.design_kernels("santa_block_kernel (twins, 4-wave code-pair tile)") == ["santa_block_kernel"]
    for blocks in (78, 466, 467, 12345):
        t = bench.stored_traffic(["santa_block_kernel"], blocks)
        if t["traffic"] is not None:
            s = json.load(open(os.path.join(root, "profiles", t["traffic_source"].split(" ")[0])))
            assert s["probe"]["blocks"] == blocks
        o = bench.stored_occupancy("santa_block_kernel", blocks)
        if o is not None:
            s = json.load(open(os.path.join(root, "profiles", o["source"].split(" ")[0])))
            assert s["probe"]["blocks"] == blocks
    assert bench.stored_traffic(["santa_block_kernel"], 12345)["traffic"] is None
    t = bench.stored_traffic(["santa_tile_kernel", "santa_sp3_kernel"], 3730)
    if t["traffic"] is None:
        assert "kernel source" in t["traffic_note"]
    else:
        raw = t["traffic_raw"]
        s = json.load(open(os.path.join(root, "profiles", t["traffic_source"].split(" ")[0])))
        hb = s["hbm_bytes_per_launch"]
        est = sum(hb[k]["FETCH_SIZE_bytes"] * f for k, f in zip(raw["kernels"], raw["fetch_correction"]))
        assert t["traffic"] == round(est + raw["WRITE_SIZE"])
        # (the fused build of round 4: the summary holds santa_sp3_kernel alone;
        # santa_tile_kernel runs only for contexts without the packed wishlists)
        assert "santa_sp3_kernel" in raw["kernels"]
        assert set(raw["kernels"]) <= {"santa_tile_kernel", "santa_sp3_kernel"}


def test_error_flags_are_described_by_bit():
    """The device error flags reach the user as what they mean (an infeasible
    solve or a bad gift type is not reported as 'rows out of range')."""
    assert _lib.describe_error_flags(0) == "none"
    assert "child ids" in _lib.describe_error_flags(_lib.SH_ERRF_ROWS)
    assert _lib.describe_error_flags(_lib.SH_ERRF_INFEASIBLE) == "an infeasible solve"
    both = _lib.describe_error_flags(_lib.SH_ERRF_TYPE | _lib.SH_ERRF_INFEASIBLE)
    assert "gift type" in both and "infeasible" in both and "child ids" not in both
    assert "unknown bits 0x10" in _lib.describe_error_flags(0x10)


def test_bench_whole_node_cpu_projection():
    """bench.py's whole-host CPU comparator: the leased-core figures scaled by
    host threads / leased threads (B1 from its largest measured P)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    cb = {"value": 100.0, "cores": 16, "reference_lap_blocks_per_s": 50.0,
          "b1_blocks_per_s": {"8": 4.0, "16": 8.0}}
    wn = bench.whole_node_cpu(cb, {"nproc": 256, "used": 16})
    assert wn["cores"] == 256 and wn["from_cores"] == 16 and wn["factor"] == 16.0
    assert wn["port_blocks_per_s"] == 1600.0 and wn["reference_lap_blocks_per_s"] == 800.0
    assert wn["b1_blocks_per_s"] == 128.0 and wn["b1_from_procs"] == 16
    # a host with no more threads than leased: the measured figures themselves
    wn = bench.whole_node_cpu(cb, {"nproc": 8, "used": 16})
    assert wn["cores"] == 16 and wn["port_blocks_per_s"] == 100.0


def test_bench_whole_node_cpu_capped_at_round_blocks():
    """Configs with fewer blocks per round than host threads (78 twins blocks,
    6 blocks of 3000 pairs): a round's blocks are its only parallelism, so the
    projected whole-host CPU uses at most that many threads, and the measured
    figure's busy threads are capped the same way."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    cb = {"value": 160.0, "cores": 16, "round_blocks": 78, "reference_lap_blocks_per_s": 32.0,
          "b1_blocks_per_s": {"8": 4.0, "16": 8.0}}
    wn = bench.whole_node_cpu(cb, {"nproc": 256, "used": 16})
    assert wn["cores"] == 78 and wn["from_cores"] == 16 and wn["round_blocks"] == 78
    assert wn["port_blocks_per_s"] == 780.0 and wn["reference_lap_blocks_per_s"] == 156.0
    assert wn["b1_blocks_per_s"] == 39.0
    # 6 blocks per round on 16 leased threads: 6 busy, no projection beyond them
    cb = {"value": 12.0, "cores": 16, "round_blocks": 6, "b1_blocks_per_s": {"6": 3.0}}
    wn = bench.whole_node_cpu(cb, {"nproc": 256, "used": 16})
    assert wn["cores"] == 6 and wn["from_cores"] == 6 and wn["port_blocks_per_s"] == 12.0
    assert wn["b1_blocks_per_s"] == 3.0
