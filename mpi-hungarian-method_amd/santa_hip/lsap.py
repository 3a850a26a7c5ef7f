"""GPU linear_sum_assignment — the inner seam of the reference.

`linear_sum_assignment(C)` is scipy's call at mpi_single.py:101 and
mpi_twins.py:104; this module mirrors its surface for square matrices
(the only shape the reference produces): same return value (row_ind,
col_ind) as int64 numpy arrays, same ValueError on NaN / -inf / infeasible
input.  Solves run on the GPU through the C-ABI batched solvers; float64
input is replayed with scipy's own float64 arithmetic, so even the
permutation on ties is scipy's.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .context import current_stream_handle, require_gpu


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


INT64_COST_LIMIT = 1 << 50  # |C| bound that keeps every SAP value < 2^62 (n <= 1024)
EXACT_INT_LIMIT = 1 << 53   # float64 holds every integer below this exactly


def solve_batched(C: torch.Tensor, with_cost: bool = True, flags: int = 0):
    """C: device tensor [B, n, n] (int64 / int32 / float64) -> (col int32 [B, n], cost [B]).

    Infeasible blocks get col = -1 (float64 with +inf only).  int64 costs
    must satisfy |C| < 2^50 (checked on the device)."""
    require_gpu()
    if C.dim() != 3 or C.shape[1] != C.shape[2]:
        raise ValueError("expected [B, n, n]")
    C = C.contiguous()
    B, n, _ = C.shape
    dev = C.device
    col = torch.empty((B, n), dtype=torch.int32, device=dev)
    s = current_stream_handle(dev)
    L = _lib.lib()
    fl = _lib.SH_COMPAT_TIEBREAK | flags
    if C.dtype == torch.int64:
        # (max / -min as Python ints: abs() wraps at INT64_MIN)
        if C.numel() and max(int(C.max()), -int(C.min())) >= INT64_COST_LIMIT:
            raise ValueError("int64 costs must satisfy |C| < 2**50; pass float64 instead")
        cost = torch.empty(B, dtype=torch.int64, device=dev) if with_cost else None
        rc = L.lsap_solve_batched_i64(_p(C), n, B, _p(col), _p(cost), fl, s)
    elif C.dtype == torch.int32:
        cost = torch.empty(B, dtype=torch.int64, device=dev) if with_cost else None
        rc = L.lsap_solve_batched_i32(_p(C), n, B, _p(col), _p(cost), fl, s)
    elif C.dtype == torch.float64:
        cost = torch.empty(B, dtype=torch.float64, device=dev) if with_cost else None
        rc = L.lsap_solve_batched_f64(_p(C), n, B, _p(col), _p(cost), fl, s)
    else:
        raise TypeError(f"unsupported dtype {C.dtype}")
    _lib.check(rc, "lsap_solve_batched")
    return col, cost


def solve_hash(seed: int, modulus: int, n: int, B: int, device: int | str = 0, with_cost: bool = True):
    """Solve B device-generated n x n matrices (sampler.hash_matrix on the host)."""
    require_gpu()
    dev = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
    col = torch.empty((B, n), dtype=torch.int32, device=dev)
    cost = torch.empty(B, dtype=torch.int64, device=dev) if with_cost else None
    rc = _lib.lib().lsap_solve_batched_hash(ctypes.c_uint64(seed), ctypes.c_int64(modulus), n, B,
                                            _p(col), _p(cost), _lib.SH_COMPAT_TIEBREAK,
                                            current_stream_handle(dev))
    _lib.check(rc, "lsap_solve_batched_hash")
    return col, cost


def linear_sum_assignment(cost_matrix, maximize: bool = False, device: int | str = 0):
    """scipy.optimize.linear_sum_assignment for one matrix, solved on the GPU.

    Square matrices only (the reference's blocks are square).  Integer
    matrices whose sums stay below 2^53 are solved in exact int64 (where
    scipy's float64 arithmetic is exact too); anything else in float64 with
    scipy's operation order, so the permutation is scipy's either way."""
    C = np.asarray(cost_matrix)
    if C.ndim != 2:
        raise ValueError("expected a matrix (2-D array), got a %r array" % (C.shape,))
    if C.shape[0] != C.shape[1]:
        raise ValueError("santa_hip solves square cost matrices only (the reference's blocks)")
    n = C.shape[0]
    if n == 0:
        return np.zeros(0, dtype=np.int64), np.zeros(0, dtype=np.int64)
    if n > _lib.SH_MAX_N:
        raise ValueError(f"n = {n} > {_lib.SH_MAX_N}")
    dev = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
    if C.dtype == np.bool_:
        C = C.astype(np.int64)
    if np.issubdtype(C.dtype, np.unsignedinteger):
        # negating an unsigned array wraps: widen first (uint64 beyond int64 -> float64)
        C = C.astype(np.int64) if (C.size == 0 or int(C.max()) <= np.iinfo(np.int64).max) \
            else C.astype(np.float64)
    # scipy solves in float64.  Integer input is solved in exact int64, which
    # makes scipy's decisions only while every value it forms is an integer
    # below 2^53 (no float64 rounding); duals and path lengths stay within a few
    # n * max|C|, so 4 (n + 1) max|C| < 2^53 is a safe bound.  The bound is
    # taken in Python ints before any negation (np.abs / -C wrap at INT64_MIN).
    # Wider ranges take the float64 replay of scipy's own arithmetic.
    if np.issubdtype(C.dtype, np.integer) and \
            (C.size == 0 or 4 * (n + 1) * max(int(C.max()), -int(C.min())) < EXACT_INT_LIMIT):
        Ci = np.ascontiguousarray(C, dtype=np.int64)
        Ct = torch.from_numpy(-Ci if maximize else Ci).to(dev)
    else:
        Cf = np.ascontiguousarray(C, dtype=np.float64)
        if maximize:
            Cf = -Cf
        if np.isnan(Cf).any() or np.isneginf(Cf).any():
            raise ValueError("matrix contains invalid numeric entries")
        Ct = torch.from_numpy(Cf).to(dev)
    col, _ = solve_batched(Ct.unsqueeze(0), with_cost=False)
    col = col[0].cpu().numpy().astype(np.int64)
    if (col < 0).any():
        raise ValueError("cost matrix is infeasible")
    return np.arange(n, dtype=np.int64), col
