"""BASELINE config 5: pure-solver sweep (n = 64..1024, batch 1..65536) on
uniform random integer costs in [0, 2^16), against scipy on the host cores.

The inner seam of the reference is `linear_sum_assignment(C)`
(mpi_single.py:101, mpi_twins.py:104).  This tool measures the batched GPU
solvers behind it:
  * `hash`     -- lsap_solve_batched_hash: costs generated on the device from
                  (seed, block, i, j) (any batch size; no input traffic);
  * `resident` -- lsap_solve_batched_i32: B x n x n int32 costs resident in
                  HBM before the timed region (only where B*n^2*4 <= 4 GB).
Parity: for every n the first PARITY instances of the hash stream are solved
by scipy on the host and compared column for column (bit-exact permutation,
ties included) and by total cost.  scipy is the reference's own LAP; it is
timed on one core and on a process pool for the CPU baseline.

Prints one JSON object per line; the summary of a run is committed under
profiles/ (r01_solver_sweep.jsonl).
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-hungarian-method_amd"))

import numpy as np  # noqa: E402

MOD = 1 << 16
SEED = 5


def _scipy_worker(args):
    n, seed, first, count = args
    from scipy.optimize import linear_sum_assignment
    from santa_hip.sampler import hash_matrix
    mats = [hash_matrix(seed, b, n, MOD) for b in range(first, first + count)]
    t0 = time.perf_counter()
    for C in mats:
        linear_sum_assignment(C)
    return count, time.perf_counter() - t0


def scipy_rate(n, seconds, procs):
    """scipy solves/s on `procs` processes (each solves its own instances)."""
    from scipy.optimize import linear_sum_assignment
    from santa_hip.sampler import hash_matrix
    C = hash_matrix(SEED, 0, n, MOD)
    t0 = time.perf_counter()
    linear_sum_assignment(C)
    one = max(time.perf_counter() - t0, 1e-5)
    per_proc = max(1, int(seconds / one))
    if procs == 1:
        cnt, dt = _scipy_worker((n, SEED, 0, per_proc))
        return cnt / dt, cnt
    with mp.get_context("spawn").Pool(procs) as pool:
        res = pool.map(_scipy_worker, [(n, SEED, p * per_proc, per_proc) for p in range(procs)])
    total = sum(c for c, _ in res)
    return total / max(dt for _, dt in res), total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="*", default=[64, 128, 256, 512, 1024])
    ap.add_argument("--batch", type=int, nargs="*", default=[1, 16, 256, 4096, 65536])
    ap.add_argument("--parity", type=int, default=64, help="instances per n checked against scipy")
    ap.add_argument("--max-est-s", type=float, default=12.0,
                    help="skip (n, B) points whose estimated GPU time exceeds this")
    ap.add_argument("--cpu-seconds", type=float, default=1.5)
    ap.add_argument("--procs", type=int, default=16)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()

    import torch
    from scipy.optimize import linear_sum_assignment
    import santa_hip.lsap as L
    from santa_hip.sampler import hash_matrix

    assert torch.cuda.is_available(), "solver_sweep needs the MI355X"
    dev = torch.device("cuda", 0)

    def timed(fn):
        fn()  # warm-up (also JIT-free: kernels are precompiled)
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1))
        return best

    for n in a.n:
        # parity: the first a.parity instances of the hash stream vs scipy
        col, cost = L.solve_hash(SEED, MOD, n, a.parity, device=0)
        col = col.cpu().numpy()
        cost = cost.cpu().numpy()
        bad = 0
        for b in range(a.parity):
            C = hash_matrix(SEED, b, n, MOD)
            _, sc = linear_sum_assignment(C)
            if not np.array_equal(col[b], sc) or int(cost[b]) != int(C[np.arange(n), sc].sum()):
                bad += 1
        cpu1, cnt1 = scipy_rate(n, a.cpu_seconds, 1)
        cpuP, cntP = scipy_rate(n, a.cpu_seconds, a.procs)
        print(json.dumps({"n": n, "parity_instances": a.parity, "parity_mismatches": bad,
                          "scipy_solves_per_s_1core": round(cpu1, 1),
                          f"scipy_solves_per_s_{a.procs}proc": round(cpuP, 1),
                          "scipy_sample": f"{cnt1} + {cntP} instances"}), flush=True)
        last = None  # (B, ms) of the previous point: time(B') ~ ms * max(1, B'/max(B, 2048))
        for B in a.batch:
            if last is not None:
                est = last[1] * max(1.0, B / max(last[0], 2048)) / 1e3
                if est > a.max_est_s:
                    print(json.dumps({"n": n, "B": B, "skipped": f"estimated {est:.1f} s > max-est-s"}),
                          flush=True)
                    continue
            ms = timed(lambda: L.solve_hash(SEED, MOD, n, B, device=0))
            last = (B, ms)
            rec = {"n": n, "B": B, "source": "hash", "ms": round(ms, 4),
                   "solves_per_s": round(B / ms * 1e3, 1)}
            if B * n * n * 4 <= (4 << 30):
                C = torch.randint(0, MOD, (B, n, n), dtype=torch.int32, device=dev)
                msr = timed(lambda: L.solve_batched(C, with_cost=True))
                rec.update({"resident_ms": round(msr, 4), "resident_solves_per_s": round(B / msr * 1e3, 1)})
                del C
            rec["vs_scipy_1core"] = round(rec["solves_per_s"] / cpu1, 1)
            rec[f"vs_scipy_{a.procs}proc"] = round(rec["solves_per_s"] / cpuP, 1)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
