"""The CPU oracle against the reference's golden vectors (no GPU).

Pins the oracle before it is trusted as the GPU path's checker:
  * lsap_cases.npz     — scipy.optimize.linear_sum_assignment's own col_ind
                         (tie-heavy ints, reals, +inf) for the SAP restatement;
  * santa_blocks.npz   — the reference's optimize_block / optimize_block_twins
                         (mpi_single.py:93-102, mpi_twins.py:93-105);
  * santa_score.json   — the reference's avg_normalized_happiness
                         (mpi_single.py:13-83) on the full synthetic instance;
  * trajectory_*.json  — the reference's my_optimizer run for 3 rounds;
  * santa_triplets.npz — triplet-unit blocks (extension: the reference only
                         asserts triplets), C from the reference's float32
                         happiness table summed as mpi_twins.py:101 does for
                         two members, solved by scipy.
"""
import hashlib

import numpy as np
import pytest

import oracle
from conftest import golden_json
from cpu_engine import CPUOracleEngine, sha
from santa_hip import _lib
from santa_hip.driver import World, run_rounds


def test_lsap_int_cases_match_scipy(lsap_cases):
    z, meta = lsap_cases
    n_checked = 0
    for m in meta:
        if m["kind"] != "int":
            continue
        C = z[f"C{m['i']}"].astype(np.int64)
        want = z[f"col{m['i']}"].astype(np.int64)
        _, got = oracle.lsap(C)
        assert np.array_equal(got, want), m
        _, got_f = oracle.lsap(C.astype(np.float64))
        assert np.array_equal(got_f, want), m
        assert int(C[np.arange(C.shape[0]), got].sum()) == m["cost"]
        n_checked += 1
    assert n_checked > 100


def test_lsap_float_cases_match_scipy(lsap_cases):
    z, meta = lsap_cases
    for m in meta:
        if not m["kind"].startswith("f64"):
            continue
        C = z[f"C{m['i']}"]
        want = z[f"col{m['i']}"].astype(np.int64)
        if m["feasible"]:
            _, got = oracle.lsap(C)
            assert np.array_equal(got, want), m
            assert C[np.arange(C.shape[0]), got].sum() == m["cost"]
        else:
            with pytest.raises(ValueError):
                oracle.lsap(C)


def test_lsap_rejects_nan_and_neginf():
    with pytest.raises(ValueError):
        oracle.lsap(np.array([[np.nan, 1.0], [1.0, 2.0]]))
    with pytest.raises(ValueError):
        oracle.lsap(np.array([[-np.inf, 1.0], [1.0, 2.0]]))


def test_lsap_empty_and_rectangular():
    r, c = oracle.lsap(np.zeros((0, 0)))
    assert r.size == 0 and c.size == 0
    from scipy.optimize import linear_sum_assignment as lsa
    rng = np.random.default_rng(3)
    for _ in range(40):
        C = rng.integers(0, 4, size=(rng.integers(1, 9), rng.integers(1, 9))).astype(float)
        a, b = lsa(C), oracle.lsap(C)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def _local_block(z, m):
    """Rebuild a block-local mini instance from the fixture's block data."""
    k = m["i"]
    n = m["n"]
    ctype = z[f"ctype{k}"]
    if m["mode"] == "single":
        wish = z[f"wish{k}"]
        types = ctype.copy()
        rows = np.arange(n, dtype=np.int32)
    else:
        w2 = z[f"wish{k}"]                      # [pairs, 2, n_wish]
        wish = w2.reshape(2 * n, -1)            # child 2i = first twin, 2i+1 second
        types = np.repeat(ctype, 2)
        rows = 2 * np.arange(n, dtype=np.int32)
    return wish, types, rows


def test_santa_blocks_cost_and_assignment(santa_blocks):
    z, meta = santa_blocks
    for m in meta:
        wish, types, rows = _local_block(z, m)
        fn = oracle.cost_single if m["mode"] == "single" else oracle.cost_twins
        C = fn(wish, types, rows, ng=1000)
        _, col = oracle.lsap(C)
        assert np.array_equal(col, z[f"col{m['i']}"].astype(np.int64)), m
        assert int(C[np.arange(m["n"]), col].sum()) == m["cost_units"], m
        # the float64 matrix the reference hands scipy is C * 2^-31 exactly
        _, col_f = oracle.lsap(C.astype(np.float64) / 2 ** 31)
        assert np.array_equal(col_f, col)


def test_triplet_blocks_cost_and_assignment(santa_triplets):
    """Triplet units: float32 ((h1 + h2) + h3), exact units, scipy's col_ind."""
    z, meta = santa_triplets
    for m in meta:
        k, n = m["i"], m["n"]
        w3 = z[f"wish{k}"]                      # [units, 3, n_wish]
        wish = w3.reshape(3 * n, -1)
        types = np.repeat(z[f"ctype{k}"], 3)
        rows = 3 * np.arange(n, dtype=np.int32)
        C = oracle.cost_triplets(wish, types, rows, ng=1000)
        assert np.array_equal(C[:, :8], z[f"cunits{k}"]), m
        _, col = oracle.lsap(C)
        assert np.array_equal(col, z[f"col{k}"].astype(np.int64)), m
        assert int(C[np.arange(n), col].sum()) == m["cost_units"], m


def test_triplet_round_keeps_units(full_data):
    """The oracle's triplet round moves whole units: afterwards every triplet
    still shares a gift and the multiset of gifts is unchanged."""
    from santa_hip import sampler as S
    tri, _ = S.family_sizes(full_data.nc)
    lo, count, nb = S.triplet_geometry(tri, 128)
    rows = S.sample_blocks(3, 0, lo, count, 3, 128, nb)
    t = full_data.types.copy()
    col, cost = oracle.round_blocks(2, full_data.wish, t, rows, ng=full_data.ng)
    assert nb == 13 and col.shape == (nb, 128)
    fam = t[:tri].reshape(-1, 3)
    assert (fam == fam[:, :1]).all()
    assert np.array_equal(np.sort(t), np.sort(full_data.types))
    assert oracle.score_sums(full_data.wish, full_data.goodkids, t)[2] == 0


def test_santa_blocks_reference_sizes(full_data):
    """The reference's own block sizes: optimize_block at block_size=2000
    (mpi_single.py:238) and optimize_block_twins at 3000 pairs
    (mpi_twins.py:244), solved by the reference in the build container
    (tests/golden/santa_blocks_large.npz); the oracle's round equals them."""
    from conftest import load_npz_cases
    z, meta = load_npz_cases("santa_blocks_large.npz")
    for m in meta:
        k, n = m["i"], m["n"]
        mode = 0 if m["mode"] == "single" else 1
        t = full_data.types.copy()
        col, cost = oracle.round_blocks(mode, full_data.wish, t, z[f"rows{k}"][None], ng=full_data.ng)
        assert np.array_equal(col[0], z[f"col{k}"].astype(np.int64)), m
        assert int(cost[0]) == m["cost_units"], m


def test_score_matches_reference(full_data):
    g = golden_json("santa_score.json")
    assert sha(full_data.wish) == g["data"]["wish_sha"], "synthetic generator drifted"
    assert sha(full_data.goodkids) == g["data"]["good_sha"]
    assert sha(full_data.types) == g["data"]["types_sha"]
    base = g["entries"][0]
    sc, sg, bt, btw = oracle.score_sums(full_data.wish, full_data.goodkids, full_data.types)
    assert (sc, sg, bt, btw) == (base["S_child"], base["S_gift"], 0, 0)
    s = oracle.score_from_sums(sc, sg, full_data.nc, full_data.ng, full_data.n_wish, full_data.n_good)
    assert s == base["score"]


def csv_digest(path) -> dict:
    data = open(path, "rb").read()
    return {"sha256": hashlib.sha256(data).hexdigest(), "bytes": len(data)}


@pytest.mark.parametrize("check", [0, None])
@pytest.mark.parametrize("mode", ["single", "twins"])
def test_trajectory_matches_reference(full_data, mode, check, tmp_path):
    """run_rounds (the product driver) on the CPU oracle engine replays the
    reference's my_optimizer: same scores, bit for bit, same states, and the
    checkpoint CSV santa_hip.data.write_submission writes after each round is
    byte-identical to the reference's own subm_best[['ChildId','GiftId']]
    .to_csv(..., index=False) of that round (mpi_single.py:177,
    mpi_twins.py:183; sha256 recorded by make_golden.py).  check = 0: the
    reference's full rescore every round (the rescored states' digests are
    compared too); None: the default delta sums (every round's score from the
    blocks' exact deltas, rescored at the last round)."""
    from santa_hip import data as D
    g = golden_json(f"trajectory_{mode}.json")
    eng = CPUOracleEngine(full_data.wish, full_data.goodkids, full_data.nq)
    import torch
    types = torch.from_numpy(full_data.types.copy())
    m = _lib.SH_MODE_SINGLE if mode == "single" else _lib.SH_MODE_TWINS
    csvs = []

    def checkpoint(st):
        p = tmp_path / f"r{st.round}.csv"
        D.write_submission(str(p), types.numpy())
        csvs.append(csv_digest(p))

    res = run_rounds(eng, types, mode=m, n=g["n"], blocks_per_round=g["P"], seed=g["seed"],
                     max_rounds=g["rounds"], world=World(), score0=g["score0"], on_round=checkpoint,
                     score_check_every=check)
    assert res.rounds == len(g["per_round"])
    assert [st.score for st in res.history] == [w["score"] for w in g["per_round"]]
    assert csvs == [w["csv"] for w in g["per_round"]]
    if check == 0:
        assert [log[2] for log in eng.score_log] == [w["types_sha"] for w in g["per_round"]]
