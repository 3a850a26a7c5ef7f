"""TEST INFRASTRUCTURE ONLY — ctypes wrapper around the CPU oracle (oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker (or the timed CPU baseline).
The product package (mpi-hungarian-method_amd/santa_hip) never imports it.

What it restates (see oracle.c for the line-level citations):
  * lsap_f64 / lsap_i64 — scipy.optimize.linear_sum_assignment (scipy 1.15.3,
    third-party, called at mpi_single.py:101 / mpi_twins.py:104), pinned by
    tests/golden/lsap_cases.npz produced by scipy itself;
  * cost_single / cost_twins — optimize_block (mpi_single.py:93-100) and
    optimize_block_twins (mpi_twins.py:93-103) cost matrices, exact int64 in
    units of 2^-31, pinned by tests/golden/santa_blocks.npz (reference
    functions run in the build container);
  * score_sums / score — avg_normalized_happiness (mpi_single.py:13-83),
    pinned by tests/golden/santa_score.json;
  * round_blocks — one block round (cost + LSAP + apply), pinned by the
    trajectory fixture tests/golden/trajectory_*.json.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

_P = ctypes.c_void_p
_I = ctypes.c_int


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_lsap_f64.argtypes = [_I, _I, _P, _P, _P]
        L.oracle_lsap_i64.argtypes = [_I, _I, _P, _P, _P]
        L.oracle_lsap_i64_batched.argtypes = [_I, _I, _P, _P, _P, _P]
        L.oracle_cost_single.argtypes = [_P, _I, _I, _P, _P, _I, _P]
        L.oracle_cost_twins.argtypes = [_P, _I, _I, _P, _P, _I, _P]
        L.oracle_cost_triplets.argtypes = [_P, _I, _I, _P, _P, _I, _P]
        L.oracle_score.argtypes = [_P, _I, _P, _I, _I, _P, _I, _I, _P]
        L.oracle_round.argtypes = [_I, _P, _I, _I, _P, _P, _I, _I, _P, _P, _P]
        for f in (L.oracle_lsap_f64, L.oracle_lsap_i64, L.oracle_lsap_i64_batched,
                  L.oracle_score, L.oracle_round):
            f.restype = _I
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def lsap(C: np.ndarray, stats: np.ndarray | None = None):
    """scipy-compatible linear_sum_assignment on a 2-D matrix.

    Returns (row_ind, col_ind) like scipy; raises ValueError on infeasible or
    invalid input like scipy does.  int64 matrices use exact int64 arithmetic,
    everything else float64.
    """
    C = np.asarray(C)
    if C.ndim != 2:
        raise ValueError("expected a matrix (2-D array)")
    transpose = C.shape[1] < C.shape[0]
    if transpose:
        C = C.T
    nr, nc = C.shape
    col = np.zeros(nr, dtype=np.int64)
    st = stats if stats is not None else np.zeros(2, dtype=np.uint64)
    if C.dtype == np.int64:
        Cc = np.ascontiguousarray(C)
        rc = lib().oracle_lsap_i64(nr, nc, _ptr(Cc), _ptr(col), _ptr(st))
    else:
        Cc = np.ascontiguousarray(C, dtype=np.float64)
        if np.isnan(Cc).any() or np.isneginf(Cc).any():
            raise ValueError("matrix contains invalid numeric entries")
        rc = lib().oracle_lsap_f64(nr, nc, _ptr(Cc), _ptr(col), _ptr(st))
    if rc == -1:
        raise ValueError("cost matrix is infeasible")
    if rc != 0:
        raise ValueError(f"oracle lsap failed ({rc})")
    if transpose:
        order = np.argsort(col)
        return col[order], order.astype(np.int64)
    return np.arange(nr, dtype=np.int64), col


def lsap_i64_batched(C: np.ndarray, stats: np.ndarray | None = None):
    """B x n x n int64 -> (col [B,n] int64, cost [B] int64)."""
    C = np.ascontiguousarray(C, dtype=np.int64)
    B, n, n2 = C.shape
    assert n == n2
    col = np.zeros((B, n), dtype=np.int64)
    cost = np.zeros(B, dtype=np.int64)
    st = stats if stats is not None else np.zeros(2, dtype=np.uint64)
    rc = lib().oracle_lsap_i64_batched(n, B, _ptr(C), _ptr(col), _ptr(cost), _ptr(st))
    if rc:
        raise ValueError(f"oracle lsap failed ({rc})")
    return col, cost


def _ng_of(wish, types, ng):
    if ng is not None:
        return int(ng)
    return int(max(int(wish.max()), int(types.max())) + 1)


def cost_single(wish: np.ndarray, types: np.ndarray, rows: np.ndarray, ng: int | None = None) -> np.ndarray:
    wish = np.ascontiguousarray(wish, dtype=np.int16)
    types = np.ascontiguousarray(types, dtype=np.int16)
    rows = np.ascontiguousarray(rows, dtype=np.int32)
    n = rows.shape[0]
    C = np.zeros((n, n), dtype=np.int64)
    lib().oracle_cost_single(_ptr(wish), wish.shape[1], _ng_of(wish, types, ng), _ptr(types),
                             _ptr(rows), n, _ptr(C))
    return C


def cost_twins(wish: np.ndarray, types: np.ndarray, rows: np.ndarray, ng: int | None = None) -> np.ndarray:
    wish = np.ascontiguousarray(wish, dtype=np.int16)
    types = np.ascontiguousarray(types, dtype=np.int16)
    rows = np.ascontiguousarray(rows, dtype=np.int32)
    n = rows.shape[0]
    C = np.zeros((n, n), dtype=np.int64)
    lib().oracle_cost_twins(_ptr(wish), wish.shape[1], _ng_of(wish, types, ng), _ptr(types),
                            _ptr(rows), n, _ptr(C))
    return C


def cost_triplets(wish: np.ndarray, types: np.ndarray, rows: np.ndarray, ng: int | None = None) -> np.ndarray:
    """Triplet units (extension of mpi_twins.py:93-103 to three members)."""
    wish = np.ascontiguousarray(wish, dtype=np.int16)
    types = np.ascontiguousarray(types, dtype=np.int16)
    rows = np.ascontiguousarray(rows, dtype=np.int32)
    n = rows.shape[0]
    C = np.zeros((n, n), dtype=np.int64)
    lib().oracle_cost_triplets(_ptr(wish), wish.shape[1], _ng_of(wish, types, ng), _ptr(types),
                               _ptr(rows), n, _ptr(C))
    return C


def family_sizes(nc: int) -> tuple[int, int]:
    """(n_triplets, n_twins) exactly as mpi_single.py:27-28 derives them."""
    import math
    twins = math.ceil(0.04 * nc / 2.) * 2
    triplets = math.ceil(0.005 * nc / 3.) * 3
    return triplets, twins


def score_sums(wish: np.ndarray, good: np.ndarray, types: np.ndarray):
    """-> (S_child, S_gift, triplet_violations, twin_violations)."""
    wish = np.ascontiguousarray(wish, dtype=np.int16)
    good = np.ascontiguousarray(good, dtype=np.int32)
    types = np.ascontiguousarray(types, dtype=np.int16)
    nc = types.shape[0]
    tri, tw = family_sizes(nc)
    out = np.zeros(4, dtype=np.int64)
    lib().oracle_score(_ptr(wish), wish.shape[1], _ptr(good), good.shape[1], nc,
                       _ptr(types), tri, tw, _ptr(out))
    return tuple(int(x) for x in out)


def score_from_sums(s_child: int, s_gift: int, nc: int, ng: int, n_wish: int, n_good: int) -> float:
    """The float tail of avg_normalized_happiness (mpi_single.py:80-81).

    np.mean over the per-gift float64 totals is exact (integers < 2**53) and
    equals S_gift / ng rounded once, so the same Python expression is used.
    """
    max_child = n_wish * 2
    max_gift = n_good * 2
    nq = nc // ng
    return (s_child / (nc * float(max_child))) ** 3 + \
        ((s_gift / ng) / float(max_gift * nq)) ** 3


def round_blocks(mode: int, wish: np.ndarray, types: np.ndarray, rows: np.ndarray,
                 stats: np.ndarray | None = None, ng: int | None = None):
    """One CPU round over B blocks (rows [B, n]); types updated in place.

    Returns (col [B,n] int64, cost [B] int64)."""
    wish = np.ascontiguousarray(wish, dtype=np.int16)
    assert types.dtype == np.int16 and types.flags.c_contiguous
    rows = np.ascontiguousarray(rows, dtype=np.int32)
    B, n = rows.shape
    col = np.zeros((B, n), dtype=np.int64)
    cost = np.zeros(B, dtype=np.int64)
    st = stats if stats is not None else np.zeros(2, dtype=np.uint64)
    rc = lib().oracle_round(mode, _ptr(wish), wish.shape[1], _ng_of(wish, types, ng), _ptr(types),
                            _ptr(rows), n, B,
                            _ptr(col), _ptr(cost), _ptr(st))
    if rc:
        raise ValueError(f"oracle round failed ({rc})")
    return col, cost
