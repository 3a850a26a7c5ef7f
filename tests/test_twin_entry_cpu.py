"""CPU check of the twins tile-entry encoding of the 4-wave twins kernel
(santa_hip.hip: twin_entry / twin_entry_cost): every code pair's entry must
decode to the cost the reference computes, float32(h1 + h2) for the two
twins' happiness values (mpi_twins.py:99-101), in units of 2^-31.  The
context runs the same check in C++ at creation (sh_ctx_create); this test
restates the encoding in Python and pins it against numpy's float32 sums for
the synthetic shape (n_wish = 100) and the small wishlists the GPU tests use."""
import numpy as np
import pytest


def miss_units(n_wish: int) -> int:
    return int(np.float64(np.float32(1.0 / (2.0 * n_wish))) * 2.0 ** 31)


def entry(c1: int, c2: int, n_wish: int, E: int) -> int:
    nw1 = n_wish + 1
    a = (nw1 - c1 if c1 else 0) + (nw1 - c2 if c2 else 0)
    if c1 and c2:
        return a | (31 << 8)
    if not (c1 or c2):
        return (1 << 8) | (1 << 14)  # k = 1 with the double bit: m = E << 1 (round 4)
    k = 39 - (32 - (2 * a - 1).bit_length())  # 39 - clz32(2a - 1)
    q = 1 << k
    rem, half = E & (q - 1), q >> 1
    base = E - rem
    up = 1 if (rem > half or (rem == half and (base >> k) & 1)) else 0
    return a | (k << 8) | (up << 13)


def decode(e: int, E: int) -> int:
    """twin_entry_cost<0> (round 4): m = ((E >> (k - dbl)) + up) << k."""
    a, t = e & 0xFF, e >> 8
    up, dbl = (t >> 5) & 1, (t >> 6) & 1
    m = (((E >> ((t - dbl) & 31)) + up) << (t & 31)) & 0xFFFFFFFF
    return m - (a << 32)


def decode_scaled(e: int, E: int, sh: int = 17) -> int:
    """twin_entry_cost<17>: the two 32-bit halves of (m - a * 2^32) << sh."""
    a, t = e & 0xFF, e >> 8
    up, dbl = (t >> 5) & 1, (t >> 6) & 1
    m = (((E >> ((t - dbl) & 31)) + up) << (t & 31)) & 0xFFFFFFFF
    lo = (m << sh) & 0xFFFFFFFF
    hi = ((m >> (32 - sh)) - (a << sh)) & 0xFFFFFFFF
    v = (hi << 32) | lo
    return v - (1 << 64) if v >> 63 else v


def decode_r3(e: int, E: int) -> int:
    """Round 3's form of the same decode: ((E & -2^k) + up * 2^k) << dbl
    (a miss pair then had k = 0)."""
    a, k, up, dbl = e & 0xFF, (e >> 8) & 31, (e >> 13) & 1, (e >> 14) & 1
    if dbl:
        k = 0
    q = (1 << k) & 0xFFFFFFFF
    m = (((E & ((0 - q) & 0xFFFFFFFF)) + up * q) << dbl) & 0xFFFFFFFF
    return m - (a << 32)


@pytest.mark.parametrize("n_wish", [100, 10, 7, 12, 126])
def test_twin_entries_decode_to_float32_sums(n_wish):
    E = miss_units(n_wish)
    miss = np.float32(1.0 / (2.0 * n_wish))
    h = [miss] + [np.float32(-2.0 * (n_wish - (c - 1))) for c in range(1, n_wish + 1)]
    for c1 in range(n_wish + 1):
        for c2 in range(n_wish + 1):
            s = np.float32(h[c1] + h[c2])  # numpy float32 add: one rounding
            want = int(np.float64(s) * 2.0 ** 31)
            e = entry(c1, c2, n_wish, E)
            assert e < 1 << 16
            assert decode(e, E) == want, (n_wish, c1, c2)
            assert decode_r3(e, E) == want, (n_wish, c1, c2)
            assert decode_scaled(e, E) == want * (1 << 17), (n_wish, c1, c2)
