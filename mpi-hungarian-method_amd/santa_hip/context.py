"""Device-resident problem state and the hot-path calls on one GPU.

`SantaGPU` replaces the module-level state of mpi_single.py:187-227 (one MPI
rank's copy of the wishlists, good-kids lists and the 4 GB dense happiness
tables): the tables live once in HBM inside a C-ABI context (sh_ctx), the
current assignment is an int16 gift-type vector [nc] on the device, and each
call below is one C-ABI launch on torch's current HIP stream.  PyTorch is
used only for device memory and streams.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .data import SantaData
from .sampler import family_sizes, single_geometry, triplet_geometry, twin_geometry


def _ptr(t: torch.Tensor | None):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _host_ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def current_stream_handle(device: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_gpu() -> None:
    if not torch.cuda.is_available():
        raise RuntimeError("santa_hip needs a ROCm GPU (torch.cuda.is_available() is False); "
                           "there is no CPU fallback")


class SantaGPU:
    """One GPU's copy of a Santa instance (one rank of the reference)."""

    def __init__(self, wish: np.ndarray, goodkids: np.ndarray, nq: int, device: int | str = 0):
        require_gpu()
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        wish = np.ascontiguousarray(wish, dtype=np.int16)
        goodkids = np.ascontiguousarray(goodkids, dtype=np.int32)
        self.nc, self.n_wish = wish.shape
        self.ng, self.n_good = goodkids.shape
        self.nq = int(nq)
        self.n_triplets, self.n_twins = family_sizes(self.nc)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            rc = _lib.lib().sh_ctx_create(ctypes.byref(h), self.device.index or 0, _host_ptr(wish),
                                          self.n_wish, _host_ptr(goodkids), self.n_good, self.nc,
                                          self.ng, self.nq)
        _lib.check(rc, "sh_ctx_create")
        self._h = h
        self._sums = torch.zeros(4, dtype=torch.int64, device=self.device)

    @classmethod
    def from_data(cls, data: SantaData, device: int | str = 0) -> "SantaGPU":
        return cls(data.wish, data.goodkids, data.nq, device)

    def close(self) -> None:
        if getattr(self, "_h", None):
            _lib.lib().sh_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- state ----------------------------------------------------------------
    def upload_types(self, types: np.ndarray) -> torch.Tensor:
        """Gift type per child -> device int16 [nc].  Every type must be in
        [0, ng): the kernels index on-chip tables with it (the reference's
        numpy indexing raises IndexError on such input)."""
        types = np.asarray(types)
        if types.shape != (self.nc,):
            raise ValueError(f"expected {self.nc} gift types, got shape {types.shape}")
        check_types(types, self.ng)
        t = torch.from_numpy(np.ascontiguousarray(types, dtype=np.int16))
        return t.to(self.device)

    @property
    def stream(self):
        return current_stream_handle(self.device)

    # -- A1 sampler -------------------------------------------------------------
    def geometry(self, mode: int, n: int) -> tuple[int, int, int, int]:
        """(lo, count, stride, n_blocks) of a full round (all disjoint blocks)."""
        if mode == _lib.SH_MODE_SINGLE:
            lo, count, nb = single_geometry(self.nc, n, self.n_triplets, self.n_twins)
            return lo, count, 1, nb
        if mode == _lib.SH_MODE_TRIPLETS:
            lo, count, nb = triplet_geometry(self.n_triplets, n)
            return lo, count, 3, nb
        lo, count, nb = twin_geometry(self.n_triplets, self.n_twins, n)
        return lo, count, 2, nb

    def sample_blocks(self, mode: int, n: int, B: int, seed: int, round_: int,
                      out: torch.Tensor | None = None) -> torch.Tensor:
        lo, count, stride, nb = self.geometry(mode, n)
        if B > nb:
            raise ValueError(f"only {nb} disjoint blocks of {n} exist, asked for {B}")
        rows = out if out is not None else torch.empty(B * n, dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):  # (no context: launches on the current device)
            rc = _lib.lib().sh_sample_blocks(ctypes.c_uint64(seed), ctypes.c_uint64(round_), lo,
                                             count, stride, n, B, _ptr(rows), self.stream)
        _lib.check(rc, "sh_sample_blocks")
        return rows

    def sample_blocks_undo(self, mode: int, n: int, B: int, seed: int, round_: int, types: torch.Tensor,
                           out: torch.Tensor, undo: torch.Tensor) -> torch.Tensor:
        """sample_blocks + the round's undo record in one launch: undo[k] =
        types[rows[k]] (the round's starting types at its rows); unpack_types(
        types, rows, undo, mode) undoes the round (sh_sample_blocks_undo)."""
        lo, count, stride, nb = self.geometry(mode, n)
        if B > nb:
            raise ValueError(f"only {nb} disjoint blocks of {n} exist, asked for {B}")
        assert out.dtype == torch.int32 and out.numel() >= B * n and out.device == self.device
        assert undo.dtype == torch.int16 and undo.numel() >= B * n and undo.device == self.device
        assert types.dtype == torch.int16 and types.numel() == self.nc and types.device == self.device
        with torch.cuda.device(self.device):
            rc = _lib.lib().sh_sample_blocks_undo(ctypes.c_uint64(seed), ctypes.c_uint64(round_), lo, count,
                                                  stride, n, B, _ptr(out), _ptr(types), _ptr(undo),
                                                  self.stream)
        _lib.check(rc, "sh_sample_blocks_undo")
        return out

    # -- A2-A6 fused block round ----------------------------------------------------
    def solve_blocks(self, mode: int, rows: torch.Tensor, n: int, types: torch.Tensor,
                     col: torch.Tensor | None = None, cost: torch.Tensor | None = None,
                     delta: torch.Tensor | None = None, steps: torch.Tensor | None = None,
                     flags: int = 0) -> None:
        """Build, solve and apply B = rows.numel() // n disjoint blocks in place
        (with SH_FLAG_NO_APPLY: solve only, types untouched, blocks may overlap)."""
        assert rows.dtype == torch.int32 and rows.is_contiguous() and rows.device == self.device
        assert types.dtype == torch.int16 and types.numel() == self.nc and types.device == self.device
        B = rows.numel() // n
        assert B * n == rows.numel()
        for t, dt, size in ((col, torch.int32, B * n), (cost, torch.int64, B),
                            (delta, torch.int64, 2), (steps, torch.int64, B)):
            if t is not None:
                assert t.dtype == dt and t.numel() >= size and t.device == self.device
        rc = _lib.lib().sh_solve_blocks(self._h, mode, _ptr(rows), n, B, _ptr(types), _ptr(col),
                                        _ptr(cost), _ptr(delta), _ptr(steps),
                                        _lib.SH_COMPAT_TIEBREAK | flags, self.stream)
        _lib.check(rc, "sh_solve_blocks")

    def solve_round(self, mode: int, rows: torch.Tensor, n: int, types: torch.Tensor,
                    undo: torch.Tensor | None = None, next_round: tuple | None = None,
                    col: torch.Tensor | None = None, cost: torch.Tensor | None = None,
                    delta: torch.Tensor | None = None, steps: torch.Tensor | None = None,
                    publish: tuple | None = None, flags: int = 0) -> None:
        """solve_blocks + the loop's round bookkeeping in the same launches
        (sh_solve_round): undo[k] = the round's starting type at rows[k];
        next_round = (seed, round, B, out) samples that round's rows into out
        (the values sample_blocks writes); publish = (slot, seq) publishes
        delta into the mailbox afterwards (publish_delta's effect)."""
        assert rows.dtype == torch.int32 and rows.is_contiguous() and rows.device == self.device
        assert types.dtype == torch.int16 and types.numel() == self.nc and types.device == self.device
        B = rows.numel() // n
        assert B * n == rows.numel()
        for t, dt, size in ((col, torch.int32, B * n), (cost, torch.int64, B), (delta, torch.int64, 2),
                            (steps, torch.int64, B), (undo, torch.int16, B * n)):
            if t is not None:
                assert t.dtype == dt and t.numel() >= size and t.device == self.device
        ext = _lib.RoundExt()
        ext.d_undo = undo.data_ptr() if undo is not None else None
        if next_round is not None:
            seed, rnd, Bn, out = next_round
            lo, count, stride, nb = self.geometry(mode, n)
            if Bn > nb:
                raise ValueError(f"only {nb} disjoint blocks of {n} exist, asked for {Bn}")
            assert out.dtype == torch.int32 and out.numel() >= Bn * n and out.device == self.device
            ext.next_rows = out.data_ptr()
            ext.next_seed, ext.next_round = seed, rnd
            ext.next_lo, ext.next_count, ext.next_stride, ext.next_B = lo, count, stride, Bn
        if publish is not None:
            assert delta is not None
            ext.publish = 1
            ext.publish_slot, ext.publish_seq = int(publish[0]), int(publish[1])
        rc = _lib.lib().sh_solve_round(self._h, mode, _ptr(rows), n, B, _ptr(types), _ptr(col), _ptr(cost),
                                       _ptr(delta), _ptr(steps), ctypes.byref(ext),
                                       _lib.SH_COMPAT_TIEBREAK | flags, self.stream)
        _lib.check(rc, "sh_solve_round")

    def solve_design(self, mode: int, n: int, B: int, flags: int = 0) -> int:
        """The kernel design (SH_DESIGN_*) solve_blocks dispatches to."""
        rc = _lib.lib().sh_solve_design(self._h, mode, n, B, _lib.SH_COMPAT_TIEBREAK | flags)
        return _lib.check(rc, "sh_solve_design")

    def resident_blocks(self, mode: int, n: int, B: int, flags: int = 0) -> int:
        """Blocks of that launch's kernel the device runs at once."""
        rc = _lib.lib().sh_resident_blocks(self._h, mode, n, B, _lib.SH_COMPAT_TIEBREAK | flags)
        return _lib.check(rc, "sh_resident_blocks")

    @property
    def mailbox(self):
        """The context's host mailbox (8 int64, read live: ctypes array over
        the coherent pinned words sh_publish_delta writes)."""
        if getattr(self, "_mail", None) is None:
            p = _lib.lib().sh_ctx_mailbox(self._h)
            self._mail = ctypes.cast(p, ctypes.POINTER(ctypes.c_int64 * 8)).contents
        return self._mail

    def publish_delta(self, delta: torch.Tensor, slot: int, seq: int) -> None:
        """Enqueue: delta[0..1] -> mailbox words 4 slot + 1, + 2, then seq ->
        word 4 slot; delta zeroed (sh_publish_delta)."""
        assert delta.dtype == torch.int64 and delta.numel() >= 2 and delta.device == self.device
        _lib.check(_lib.lib().sh_publish_delta(self._h, _ptr(delta), int(slot), int(seq), self.stream),
                   "sh_publish_delta")

    def error_flags(self) -> int:
        return _lib.check(_lib.lib().sh_ctx_error_flags(self._h, self.stream), "sh_ctx_error_flags")

    def set_sparse_budget(self, nbytes: int) -> int:
        """LDS bytes per block of the default singles kernel (0 = default);
        returns the per-block hit-list capacity.  Blocks over it are solved by
        the register-tile fallback launch (same results)."""
        return _lib.check(_lib.lib().sh_ctx_set_sparse_budget(self._h, int(nbytes)),
                          "sh_ctx_set_sparse_budget")

    def fallback_steps(self) -> int:
        """Steps since the last call that used the exact two-pass argmin."""
        return _lib.check(_lib.lib().sh_ctx_fallback_steps(self._h, self.stream),
                          "sh_ctx_fallback_steps")

    # -- A7 score ---------------------------------------------------------------
    def score_sums_async(self, types: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        out = out if out is not None else self._sums
        rc = _lib.lib().sh_score(self._h, _ptr(types), _ptr(out), self.stream)
        _lib.check(rc, "sh_score")
        return out

    def score_sums(self, types: torch.Tensor) -> tuple[int, int, int, int]:
        s = self.score_sums_async(types).cpu().tolist()
        return tuple(int(x) for x in s)

    def score(self, types: torch.Tensor, check_families: bool = True) -> float:
        sc, sg, bad_tri, bad_tw = self.score_sums(types)
        if check_families and (bad_tri or bad_tw):
            raise AssertionError(f"{bad_tri} triplets / {bad_tw} twin pairs do not share a gift "
                                 "(mpi_single.py:32-44)")
        return score_from_sums(sc, sg, self.nc, self.ng, self.n_wish, self.n_good)

    # -- exchange helpers (multi-GPU) ---------------------------------------------
    def pack_types(self, types: torch.Tensor, rows: torch.Tensor, out: torch.Tensor) -> None:
        with torch.cuda.device(self.device):
            rc = _lib.lib().sh_pack_types(_ptr(types), _ptr(rows), rows.numel(), _ptr(out),
                                          self.stream)
        _lib.check(rc, "sh_pack_types")

    def unpack_types(self, types: torch.Tensor, rows: torch.Tensor, vals: torch.Tensor,
                     mode: int) -> None:
        with torch.cuda.device(self.device):
            rc = _lib.lib().sh_unpack_types(_ptr(types), _ptr(rows), rows.numel(), _ptr(vals), mode,
                                            self.stream)
        _lib.check(rc, "sh_unpack_types")


def check_types(types: np.ndarray, ng: int) -> None:
    """Reject gift types outside [0, ng) (a missing child is -1)."""
    if types.size:
        lo, hi = int(types.min()), int(types.max())
        if lo < 0 or hi >= ng:
            bad = int(np.flatnonzero((types < 0) | (types >= ng))[0])
            raise ValueError(f"gift type {int(types[bad])} of child {bad} is outside [0, {ng})")


def score_from_sums(s_child: int, s_gift: int, nc: int, ng: int, n_wish: int, n_good: int) -> float:
    """Float tail of avg_normalized_happiness (mpi_single.py:80-81).

    The per-gift totals are integers, so np.mean over them is S_gift / ng
    rounded once; the expression is the reference's own."""
    max_child_happiness = n_wish * 2
    max_gift_happiness = n_good * 2
    n_gift_quantity = nc // ng
    return (s_child / (nc * float(max_child_happiness))) ** 3 + \
        ((s_gift / ng) / float(max_gift_happiness * n_gift_quantity)) ** 3
