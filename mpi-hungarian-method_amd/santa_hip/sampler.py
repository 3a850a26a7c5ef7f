"""Block sampler and hash costs — host mirror of csrc/sh_common.h (numpy uint64).

The reference draws `np.random.permutation(range(lo, hi))` and `np.split`s it
into equal blocks each round, unseeded (mpi_single.py:118,123-124;
mpi_twins.py:125-126).  The build replaces that with a keyed 4-round Feistel
bijection of [0, count) + cycle walking, evaluated per index on the GPU
(sh_sample_blocks); this module computes the same permutation on the host so
that tests and the multi-rank driver can reproduce any round's blocks.
"""
from __future__ import annotations

import math

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def mix2(a, b):
    return splitmix64(np.asarray(a, dtype=np.uint64) ^ splitmix64(b))


class Feistel:
    """Keyed bijection of [0, count); identical to sh_feistel_* in C."""

    def __init__(self, seed: int, round_: int, count: int):
        bits = 2
        while (1 << bits) < count:
            bits += 1
        if bits & 1:
            bits += 1
        self.half = np.uint64(bits // 2)
        self.mask = np.uint64((1 << (bits // 2)) - 1)
        self.count = int(count)
        base = mix2(np.uint64(seed), np.uint64(round_) ^ np.uint64(0x5851F42D4C957F2D))
        with np.errstate(over="ignore"):
            self.keys = [splitmix64(base + np.uint64(r)) for r in range(4)]

    def encrypt(self, x: np.ndarray) -> np.ndarray:
        L = x >> self.half
        R = x & self.mask
        for k in self.keys:
            t = L ^ (splitmix64(R ^ k) & self.mask)
            L, R = R, t
        return (L << self.half) | R

    def perm(self, idx) -> np.ndarray:
        y = self.encrypt(np.asarray(idx, dtype=np.uint64))
        bad = y >= np.uint64(self.count)
        while bad.any():
            y[bad] = self.encrypt(y[bad])
            bad = y >= np.uint64(self.count)
        return y.astype(np.int64)


def single_geometry(nc: int, block_size: int, n_triplets: int, n_twins: int):
    """(lo, count, n_blocks) of the singles sampler, mpi_single.py:123-124,238-240.

    The reference permutes range(tts, n_children - children_rmd) with
    n_blocks = (n_children - tts) // block_size."""
    tts = n_triplets + n_twins
    n_blocks = (nc - tts) // block_size
    return tts, n_blocks * block_size, n_blocks


def twin_geometry(n_triplets: int, n_twins: int, pairs: int):
    """(lo, count, n_blocks) for twins, mpi_twins.py:125-126,244-246.

    block_size there counts children (2 per pair): n_blocks =
    twins // block_size, twins_rmd = twins - n_blocks*block_size, first-twin
    ids range(triplets, tts - twins_rmd, 2)."""
    block_size = 2 * pairs
    n_blocks = n_twins // block_size
    return n_triplets, n_blocks * pairs, n_blocks


def triplet_geometry(n_triplets: int, units: int):
    """(lo, count, n_blocks) for triplet blocks (an extension: the reference
    never moves triplets, it asserts they share a gift, mpi_single.py:32-37).
    Units are first-triplet ids 0, 3, ..., n_triplets - 3 (mpi_single.py:27-28
    puts the triplets first); a block holds `units` of them."""
    count = n_triplets // 3
    return 0, count, count // units


def sample_blocks(seed: int, round_: int, lo: int, count: int, stride: int, n: int, B: int) -> np.ndarray:
    """Host mirror of sh_sample_blocks -> int32 [B, n] row ids."""
    if B * n > count:
        raise ValueError("B * n exceeds the eligible count")
    f = Feistel(seed, round_, count)
    p = f.perm(np.arange(B * n, dtype=np.uint64))
    return (lo + stride * p).astype(np.int32).reshape(B, n)


def hash_cost(seed: int, b, i, j, modulus: int) -> np.ndarray:
    """Host mirror of sh_hash_cost(...) % modulus (device-generated LSAP costs)."""
    b = np.asarray(b, dtype=np.uint64)
    i = np.asarray(i, dtype=np.uint64)
    j = np.asarray(j, dtype=np.uint64)
    x = (b << np.uint64(40)) ^ (i << np.uint64(20)) ^ j
    h = splitmix64(np.uint64(seed) ^ splitmix64(x))
    return (h % np.uint64(modulus)).astype(np.int64)


def hash_matrix(seed: int, b: int, n: int, modulus: int) -> np.ndarray:
    ii, jj = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    return hash_cost(seed, b, ii, jj, modulus)


def family_sizes(nc: int) -> tuple[int, int]:
    """(n_triplets, n_twins) exactly as mpi_single.py:27-28 derives them."""
    twins = math.ceil(0.04 * nc / 2.) * 2
    triplets = math.ceil(0.005 * nc / 3.) * 3
    return triplets, twins
