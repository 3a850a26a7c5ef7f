"""BASELINE config 2 as a pure-solver figure: 4096 Santa-shaped n=256 tiles
through the batched int64 LSAP (lsap_solve_batched_i64), the reference's
linear_sum_assignment seam (mpi_single.py:101) with costs already in HBM.

The tiles are the singles blocks of rounds 0 and 1 (3730 + 366 blocks; a
round has only 3730 disjoint blocks, so 4096 tiles span two samplings) with
C[i][j] = the reference's child_happiness[child_i][type_j]
(mpi_single.py:213-218) in exact units of 2^-31, built on the GPU with torch
(tool code, not the product path).  Checks: the first --check tiles are
rebuilt by the CPU oracle (oracle.cost_single) and solved by it; col and cost
must agree bit for bit.  scipy (the reference's LAP) on one core gives the
CPU figure for the same tiles.

The same 4096 blocks also go through the fused Santa path (sh_solve_blocks:
tile build from the wishlists + scipy-exact solve, BASELINE config 2 as
stated: 4096 n=256 blocks in one batch) with SH_FLAG_NO_APPLY, since blocks
of two samplings overlap and may not both write the gift types.

Prints one JSON line (committed as profiles/<tag>_santa_tiles.json).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-hungarian-method_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", type=int, default=4096)
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--check", type=int, default=24)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--scipy-tiles", type=int, default=40)
    a = ap.parse_args()

    import torch
    import oracle
    import santa_hip.lsap as L
    from santa_hip import data as D
    from santa_hip.sampler import sample_blocks, single_geometry
    from scipy.optimize import linear_sum_assignment

    assert torch.cuda.is_available(), "santa_tiles needs the MI355X"
    dev = torch.device("cuda", 0)
    sd = D.synthetic(2017)
    n, T = a.n, a.tiles
    tri, tw = sd.families
    lo, count, nb = single_geometry(sd.nc, n, tri, tw)
    rows = []
    rnd = 0
    while sum(r.shape[0] for r in rows) < T:
        rows.append(sample_blocks(2017, rnd, lo, count, 1, n, nb))
        rnd += 1
    rows = np.concatenate(rows)[:T]                                   # [T, n] child ids

    # -- cost tiles on the GPU: C[b, i, j] = happiness(child_bi, type of child_bj)
    nw, ng = sd.n_wish, sd.ng
    E = int(round(float(np.float32(1.0 / (2 * nw))) * 2 ** 31))
    wish = torch.from_numpy(sd.wish.astype(np.int64)).to(dev)
    types = torch.from_numpy(sd.types.astype(np.int64)).to(dev)
    vals = ((torch.arange(nw, device=dev) - nw) * (1 << 32)).to(torch.int64)  # rank r: -(nw - r) * 2^32
    C = torch.empty((T, n, n), dtype=torch.int64, device=dev)
    rows_d = torch.from_numpy(rows.astype(np.int64)).to(dev)
    ch = 256
    for b0 in range(0, T, ch):
        r = rows_d[b0:b0 + ch]                                        # [c, n]
        c = r.shape[0]
        tab = torch.full((c * n, ng), E, dtype=torch.int64, device=dev)
        w = wish[r.reshape(-1)]                                       # [c*n, nw]
        # the reference's loop order: later ranks overwrite earlier ones
        for k in range(nw):
            tab[torch.arange(c * n, device=dev), w[:, k]] = vals[k]
        ct = types[r]                                                 # [c, n] column types
        C[b0:b0 + c] = tab.view(c, n, ng).gather(2, ct[:, None, :].expand(c, n, n))
        del tab, w
    torch.cuda.synchronize()

    # -- the batched solver on the resident tiles
    col, cost = L.solve_batched(C)
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        col, cost = L.solve_batched(C)
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    colh, costh = col.cpu().numpy(), cost.cpu().numpy()

    # -- the fused Santa path on the same 4096 blocks (no apply: they overlap)
    from santa_hip import _lib
    from santa_hip.context import SantaGPU
    ctx = SantaGPU.from_data(sd, 0)
    tdev = ctx.upload_types(sd.types)
    rows_f = torch.from_numpy(rows.reshape(-1).astype(np.int32)).to(dev)
    fcol = torch.empty(T * n, dtype=torch.int32, device=dev)
    fcost = torch.empty(T, dtype=torch.int64, device=dev)
    ctx.solve_blocks(0, rows_f, n, tdev, col=fcol, cost=fcost, flags=_lib.SH_FLAG_NO_APPLY)
    torch.cuda.synchronize()
    fbest = float("inf")
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ctx.solve_blocks(0, rows_f, n, tdev, col=fcol, cost=fcost, flags=_lib.SH_FLAG_NO_APPLY)
        e1.record()
        torch.cuda.synchronize()
        fbest = min(fbest, e0.elapsed_time(e1))
    assert np.array_equal(tdev.cpu().numpy(), sd.types), "SH_FLAG_NO_APPLY wrote the gift types"
    assert ctx.error_flags() == 0
    fcolh = fcol.cpu().numpy().reshape(T, n)
    fcosth = fcost.cpu().numpy()
    design = _lib.SH_DESIGN_NAMES[ctx.solve_design(0, n, T)]

    # -- oracle spot check (rebuilt on the CPU from the same rows)
    bad = 0
    for b in range(a.check):
        Cb = oracle.cost_single(sd.wish, sd.types, rows[b], ng=ng)
        assert np.array_equal(Cb, C[b].cpu().numpy()), f"tile {b}: GPU-built C differs from the oracle's"
        _, oc = oracle.lsap(Cb)
        if not np.array_equal(oc, colh[b].astype(np.int64)) or int(Cb[np.arange(n), oc].sum()) != int(costh[b]):
            bad += 1
        if not np.array_equal(oc, fcolh[b].astype(np.int64)) or int(Cb[np.arange(n), oc].sum()) != int(fcosth[b]):
            bad += 1
    # -- scipy on one core over the first tiles (float64 matrices as the reference passes)
    mats = [C[b].cpu().numpy().astype(np.float64) / 2 ** 31 for b in range(a.scipy_tiles)]
    t0 = time.perf_counter()
    for M in mats:
        linear_sum_assignment(M)
    sc_s = (time.perf_counter() - t0) / len(mats)
    out = {"workload": f"{T} Santa-shaped n={n} tiles (singles blocks of rounds 0..{rnd - 1}), "
                       "int64 costs resident in HBM, lsap_solve_batched_i64",
           "tiles": T, "n": n, "ms": round(best, 3), "tiles_per_s": round(T / best * 1e3, 1),
           "oracle_checked": a.check, "oracle_mismatches": bad,
           "scipy_tiles_per_s_1core": round(1.0 / sc_s, 1), "scipy_sample": f"{len(mats)} tiles",
           "input_bytes": int(C.numel() * 8),
           "achieved_input_GBs": round(C.numel() * 8 / best / 1e6, 1),
           "fused": {"what": "the same 4096 blocks through sh_solve_blocks (tile build from the wishlists "
                             "+ solve, SH_FLAG_NO_APPLY: the blocks of two samplings overlap)",
                     "design": design, "ms": round(fbest, 3), "blocks_per_s": round(T / fbest * 1e3, 1),
                     "oracle_checked": a.check}}
    print(json.dumps(out), flush=True)
    return 0 if bad == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
