"""TEST INFRASTRUCTURE ONLY: a CPU engine for santa_hip.driver.run_rounds built
on the oracle, so that the driver's host logic (sharding, all-gather
exchange, accept/rollback, patience) can be tested without a GPU and over
gloo.  The product engine is santa_hip.driver.GPUEngine."""
from __future__ import annotations

import hashlib

import numpy as np
import torch

import oracle
from santa_hip import _lib
from santa_hip.context import score_from_sums
from santa_hip.sampler import family_sizes, sample_blocks, single_geometry, triplet_geometry, twin_geometry


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


class CPUOracleEngine:
    def __init__(self, wish, goodkids, nq):
        self.wish = np.ascontiguousarray(wish, dtype=np.int16)
        self.good = np.ascontiguousarray(goodkids, dtype=np.int32)
        self.nc, self.n_wish = self.wish.shape
        self.ng, self.n_good = self.good.shape
        self.nq = nq
        self.n_triplets, self.n_twins = family_sizes(self.nc)
        self.score_log = []  # (S_child, S_gift, types sha) of every scored state
        self.prefetched = []  # rounds passed to prefetch_blocks
        self.drained = 0  # run_rounds' end-of-run drain() calls
        self.undo_tokens = 0  # rounds sampled with an undo record (sample_round)

    def geometry(self, mode, n):
        if mode == _lib.SH_MODE_SINGLE:
            lo, count, nb = single_geometry(self.nc, n, self.n_triplets, self.n_twins)
            return lo, count, 1, nb
        if mode == _lib.SH_MODE_TRIPLETS:
            lo, count, nb = triplet_geometry(self.n_triplets, n)
            return lo, count, 3, nb
        lo, count, nb = twin_geometry(self.n_triplets, self.n_twins, n)
        return lo, count, 2, nb

    def sample_blocks(self, mode, n, B, seed, rnd):
        lo, count, stride, _ = self.geometry(mode, n)
        return torch.from_numpy(sample_blocks(seed, rnd, lo, count, stride, n, B).reshape(-1).copy())

    def sample_round(self, mode, n, B, seed, rnd, types):
        """GPUEngine.sample_round (the undo protocol): the rows and a token
        whose undo(types) restores the round's starting types at its rows (all
        members of a unit)."""
        rows = self.sample_blocks(mode, n, B, seed, rnd)
        r = rows.numpy()
        saved = types.numpy()[r].copy()
        self.undo_tokens += 1

        class _Undo:
            def undo(_, t):
                tt = t.numpy()
                for m in range(mode + 1):
                    tt[r + m] = saved
        return rows, _Undo()

    def prefetch_blocks(self, mode, n, B, seed, rnd):
        """GPUEngine.prefetch_blocks (the exchange's `during` hook): nothing to
        prefetch on the host; its presence runs the async all-gather path."""
        self.prefetched.append(rnd)

    def drain(self):
        """GPUEngine.drain: nothing runs asynchronously on the host."""
        self.drained += 1

    def solve_blocks(self, mode, rows, n, types, delta=None):
        t = types.numpy()
        s0 = oracle.score_sums(self.wish, self.good, t) if delta is not None else None
        oracle.round_blocks(mode, self.wish, t, rows.numpy().reshape(-1, n), ng=self.ng)
        if delta is not None:  # only this engine's blocks changed in between
            s1 = oracle.score_sums(self.wish, self.good, t)
            delta += torch.tensor([s1[0] - s0[0], s1[1] - s0[1]], dtype=torch.int64)

    def new_delta(self):
        return torch.zeros(2, dtype=torch.int64)

    def delta_begin(self, types, d, full, after=None, snapshot=True):
        """Delta-round protocol (GPUEngine.delta_begin; the host copy is the
        snapshot whatever `snapshot` says)."""
        if after is not None:
            after.wait()  # (d's all-reduce)
        snap = types.clone()
        eng = self
        dv = (int(d[0]), int(d[1]))

        class _Handle:
            def result(_):
                return dv[0], dv[1], (eng.score_sums(snap) if full else None)

            def restore(_, t):
                t.copy_(snap)
        return _Handle()

    def pack_types(self, types, rows, out):
        r = rows.numpy()
        out.numpy()[:r.shape[0]] = np.where(r >= 0, types.numpy()[np.maximum(r, 0)], -1)

    def unpack_types(self, types, rows, vals, mode):
        r = rows.numpy()
        v = vals.numpy()
        m = r >= 0
        t = types.numpy()
        for k in range(mode + 1):
            t[r[m] + k] = v[m]

    def score_sums(self, types):
        t = types.numpy()
        s = oracle.score_sums(self.wish, self.good, t)
        self.score_log.append((s[0], s[1], sha(t)))
        return s

    def score_begin(self, types):
        """Pipelined-round protocol (GPUEngine.score_begin): score a snapshot."""
        snap = types.clone()
        eng = self

        class _Handle:
            def result(_):
                return eng.score_sums(snap)

            def restore(_, t):
                t.copy_(snap)
        return _Handle()

    def score_from_sums(self, sc, sg):
        return score_from_sums(sc, sg, self.nc, self.ng, self.n_wish, self.n_good)
