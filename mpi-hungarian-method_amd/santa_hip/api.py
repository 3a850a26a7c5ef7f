"""Drop-in mirrors of the reference's hot-path callables, on the GPU.

The reference exposes three module-level functions whose side inputs are
module globals:
  avg_normalized_happiness(pred, child_pref, gift_pref)   mpi_single.py:13-83
  optimize_block(child_block, current_gift_ids)           mpi_single.py:93-102
  optimize_block_twins(child_block, subm)                 mpi_twins.py:93-105
and the triplet extension optimize_block_triplets(child_block, subm).
`init(child_data, gift_data)` plays the role of the module set-up
(mpi_single.py:193-220): it uploads the tables once into a SantaGPU context
that the three functions then use, exactly as the reference's functions read
`child_happiness`, `gift_ids` and `block_size` from globals.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .context import SantaGPU, score_from_sums

_session: SantaGPU | None = None
_score_cache: dict = {}


def init(child_data: np.ndarray, gift_data: np.ndarray, n_gift_quantity: int | None = None,
         device: int | str = 0) -> SantaGPU:
    """Module set-up: child_data = wishlists [nc, 100], gift_data = good-kids [ng, 1000]."""
    global _session
    nc = child_data.shape[0]
    ng = gift_data.shape[0]
    nq = n_gift_quantity if n_gift_quantity is not None else nc // ng
    if _session is not None:
        _session.close()
    _session = SantaGPU(child_data, gift_data, nq, device)
    return _session


def session() -> SantaGPU:
    if _session is None:
        raise RuntimeError("call santa_hip.init(child_data, gift_data) first "
                           "(the reference builds these tables at module import)")
    return _session


def _types_from_pred(pred: np.ndarray, nc: int) -> np.ndarray:
    pred = np.asarray(pred)
    types = np.full(nc, -1, dtype=np.int64)  # int64: out-of-range gifts raise, not wrap
    types[pred[:, 0].astype(np.int64)] = pred[:, 1]
    if (types < 0).any():
        raise ValueError("pred must assign a gift to every child")
    return types


def avg_normalized_happiness(pred, child_pref, gift_pref) -> float:
    """Score of a full assignment, same call convention as the reference.

    As at mpi_single.py:157/233 the caller passes child_pref = gift_data
    (good-kids lists) and gift_pref = child_data (wishlists).  Raises
    AssertionError when a triplet or twin pair does not share a gift
    (mpi_single.py:32-44)."""
    good = np.asarray(child_pref)
    wish = np.asarray(gift_pref)
    s = _session
    if s is None or s.nc != wish.shape[0] or s.ng != good.shape[0]:
        key = (id(child_pref), id(gift_pref), wish.shape, good.shape)
        s = _score_cache.get(key)
        if s is None:
            _score_cache.clear()
            s = SantaGPU(wish, good, wish.shape[0] // good.shape[0])
            _score_cache[key] = s
    types = s.upload_types(_types_from_pred(pred, s.nc))
    sc, sg, bad_tri, bad_tw = s.score_sums(types)
    if bad_tri or bad_tw:
        raise AssertionError("triplets/twins must share a gift")
    return score_from_sums(sc, sg, s.nc, s.ng, s.n_wish, s.n_good)


def _solve_one(mode: int, rows: np.ndarray, types_np: np.ndarray) -> np.ndarray:
    s = session()
    n = rows.shape[0]
    if n > _lib.SH_MAX_N_SANTA:
        raise ValueError(f"block of {n} rows > {_lib.SH_MAX_N_SANTA}")
    rows_t = torch.from_numpy(np.ascontiguousarray(rows, dtype=np.int32)).to(s.device)
    types = s.upload_types(types_np)
    col = torch.empty(n, dtype=torch.int32, device=s.device)
    s.solve_blocks(mode, rows_t, n, types, col=col)
    flags = s.error_flags()
    if flags:
        raise ValueError(f"block not solved: {_lib.describe_error_flags(flags)} (device flags {flags:#x})")
    return col.cpu().numpy().astype(np.int64)


def optimize_block(child_block, current_gift_ids):
    """mpi_single.py:93-102: -> (child_block[row_ind], gift_block[col_ind]).

    current_gift_ids holds slot ids (GiftId * n_gift_quantity + rank), as
    the reference's; the cost depends only on gift types = slot // nq."""
    s = session()
    child_block = np.asarray(child_block)
    current_gift_ids = np.asarray(current_gift_ids)
    gift_block = current_gift_ids[child_block]
    types = current_gift_ids.astype(np.int64) // s.nq  # range-checked by upload_types
    col = _solve_one(_lib.SH_MODE_SINGLE, child_block, types)
    return child_block, gift_block[col]


def optimize_block_twins(child_block, subm):
    """mpi_twins.py:93-105: rows are first twins c (pairs c, c+1); columns take
    the first twin's GiftId.  -> (child_block[row_ind], gift_block[col_ind])."""
    s = session()
    child_block = np.asarray(child_block).astype(np.int64)
    gifts = subm["GiftId"].to_numpy() if hasattr(subm, "columns") else np.asarray(subm)
    gift_block = gifts[child_block]
    col = _solve_one(_lib.SH_MODE_TWINS, child_block, gifts.astype(np.int64))
    return child_block, gift_block[col]


def optimize_block_triplets(child_block, subm):
    """Triplet extension of optimize_block_twins (mpi_twins.py:93-105 with
    three members): rows are first triplets c (units c, c+1, c+2), columns
    take the first triplet's GiftId, C[i, j] = float32((h(c) + h(c+1)) +
    h(c+2)).  The reference never optimises triplets (it only asserts that
    they share a gift, mpi_single.py:32-37).
    -> (child_block[row_ind], gift_block[col_ind])."""
    s = session()
    child_block = np.asarray(child_block).astype(np.int64)
    gifts = subm["GiftId"].to_numpy() if hasattr(subm, "columns") else np.asarray(subm)
    gift_block = gifts[child_block]
    col = _solve_one(_lib.SH_MODE_TRIPLETS, child_block, gifts.astype(np.int64))
    return child_block, gift_block[col]
