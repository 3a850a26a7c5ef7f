"""Dev: a schedule model of full singles rounds on one MI355X, from the
per-block Dijkstra step counts of tools/steps_oracle.py.

Model: 1024 SIMDs x 4 resident one-wave blocks; a wave on a SIMD with k
resident waves advances one Dijkstra step every max(L, k * c) cycles (L: the
lone-step latency, c: the issue cost of one step at full occupancy).  Two
schedules:
  rounds    -- one launch per round, every block dispatched at the launch
               (block b on SIMD b mod 1024), the round ends with its last block
  dataflow  -- a block of round r+1 may start once the round-r blocks holding
               its children have finished (the only blocks it depends on),
               into any free slot, in (round, block) order
Prints the modelled time per round for both."""
import argparse
import os

import numpy as np

ap = argparse.ArgumentParser()
ap.add_argument("--npz", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                              "gpurun_out", "steps_oracle_20.npz"))
ap.add_argument("--rounds", type=int, default=20)
ap.add_argument("--L", type=float, default=1100.0)
ap.add_argument("--c", type=float, default=384.0)
ap.add_argument("--build", type=float, default=0.17e-3, help="per-round build time (rounds schedule), s")
ap.add_argument("--build-steps", type=float, default=40.0, help="per-block build cost in steps (dataflow)")
ap.add_argument("--clock", type=float, default=2.4e9)
ap.add_argument("--simds", type=int, default=1024)
ap.add_argument("--slots", type=int, default=4)
args = ap.parse_args()

z = np.load(args.npz)
R = args.rounds
rows = [z[f"rows{r}"] for r in range(R)]
steps = [z[f"steps{r}"].astype(np.float64) for r in range(R)]
B, n = rows[0].shape
S, K = args.simds, args.slots


def cyc(k):
    return np.maximum(args.L, k * args.c)


def run_round(st):
    """one launch: block b on SIMD b % S; returns the time of the last block (cycles)"""
    t_end = 0.0
    for s in range(S):
        rem = np.sort(st[s::S])
        if rem.size == 0:
            continue
        t = 0.0
        done = 0.0
        k = rem.size
        for x in rem:  # processor sharing: the shortest finishes first
            dt = (x - done) * cyc(k)
            t += dt
            done = x
            k -= 1
        t_end = max(t_end, t)
    return t_end


def run_dataflow():
    nc = int(max(r.max() for r in rows)) + 1
    # dependencies: round-r block of each child
    ready_dep = []
    for r in range(1, R):
        owner = np.empty(nc, dtype=np.int64)
        owner[rows[r - 1].ravel()] = np.repeat(np.arange(B), n)
        ready_dep.append(owner[rows[r]])  # [B, n] round-(r-1) blocks of round r's children
    total = R * B
    fin = np.full(total, np.inf)
    start = np.full(total, np.inf)
    # slots
    slot_blk = np.full(S * K, -1, dtype=np.int64)
    slot_rem = np.zeros(S * K)
    simd_of = np.arange(S * K) // K
    nxt = 0  # next block in (round, block) order to place
    t = 0.0
    dep_max = [None] + [None] * (R - 1)
    work = np.concatenate(steps) + args.build_steps
    finished = 0
    while finished < total:
        # place ready blocks in order while slots are free
        while nxt < total:
            r, b = divmod(nxt, B)
            if r > 0:
                if dep_max[r] is None:
                    dep_max[r] = np.full(B, np.nan)
                if np.isnan(dep_max[r][b]):
                    f = fin[(r - 1) * B + ready_dep[r - 1][b]]
                    if np.isinf(f).any():
                        break
                    dep_max[r][b] = f.max()
                if dep_max[r][b] > t:
                    break
            free = np.flatnonzero(slot_blk < 0)
            if free.size == 0:
                break
            occ = np.bincount(simd_of[slot_blk >= 0], minlength=S)
            cand = free[np.argmin(occ[simd_of[free]])]
            slot_blk[cand] = nxt
            slot_rem[cand] = work[nxt]
            start[nxt] = t
            nxt += 1
        act = slot_blk >= 0
        occ = np.bincount(simd_of[act], minlength=S)
        per = cyc(occ[simd_of])
        dt_fin = np.where(act, slot_rem * per, np.inf)
        i = int(np.argmin(dt_fin))
        dt = dt_fin[i]
        # the next block's dependency time may come earlier
        if nxt < total:
            r, b = divmod(nxt, B)
            if r > 0 and dep_max[r] is not None and not np.isnan(dep_max[r][b]) and dep_max[r][b] > t:
                dt = min(dt, dep_max[r][b] - t)
        slot_rem = np.where(act, slot_rem - dt / per, slot_rem)
        t += dt
        doneslots = np.flatnonzero(act & (slot_rem <= 1e-9))
        for sl in doneslots:
            fin[slot_blk[sl]] = t
            slot_blk[sl] = -1
            finished += 1
    return fin.reshape(R, B).max(axis=1)


tr = np.array([run_round(steps[r]) for r in range(R)]) / args.clock + args.build
print("rounds:   per round ms", np.round(tr * 1e3, 3).tolist())
print(f"rounds:   total {tr.sum() * 1e3:.2f} ms, mean {tr.mean() * 1e3:.3f} ms/round")
fd = run_dataflow() / args.clock
print("dataflow: round ends ms", np.round(fd * 1e3, 3).tolist())
print(f"dataflow: total {fd[-1] * 1e3:.2f} ms, mean {fd[-1] / R * 1e3:.3f} ms/round")
tot = sum(s.sum() for s in steps)
print(f"throughput floor (all slots busy): {tot * args.c * K / K / S / args.clock * 1e3:.2f} ms")
