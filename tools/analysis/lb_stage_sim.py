"""dev: how often would a wave's next candidate already be staged?

Replays scipy's SAP (numpy, same remaining order and tie rule) on one n = 2000
singles block of the bench's round 0 and, with the columns split over NW waves
as santa_lb_kernel splits them, counts per step whether the row the next step
relaxes was (a) the winning wave's previously staged best (impossible: it was
removed), (b) that wave's second-best of the previous step (top-2 staging), or
(c) neither (a dependent row load on the step's chain)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mpi-hungarian-method_amd"))
from santa_hip import data as D  # noqa: E402
from santa_hip.sampler import sample_blocks, single_geometry  # noqa: E402


def main(n=2000, NW=8, K=4, block=0):
    sd = D.synthetic(2017)
    lo, count, nb = single_geometry(sd.nc, n, *sd.families)
    rows = sample_blocks(2017, 0, lo, count, 1, n, nb)[block]
    types = sd.types[rows]
    nw = sd.n_wish
    # lattice costs (base 256): wish -a * 256, miss 1
    C = np.ones((n, n), dtype=np.int64)
    for i, c in enumerate(rows):
        rk = {int(g): r for r, g in enumerate(sd.wish[c])}
        a = np.array([nw - rk[t] if t in rk else 0 for t in types])
        C[i] = np.where(a > 0, -a * 256, 1)
    wave_of = (np.arange(n) // 64) // K
    u = np.zeros(n, np.int64)
    v = np.zeros(n, np.int64)
    r4c = -np.ones(n, np.int64)
    c4r = -np.ones(n, np.int64)
    stats = dict(steps=0, second_hit=0, top3_hit=0, improved_by_new_row=0)
    t0 = time.time()
    for cur in range(n):
        remaining = list(range(n - 1, -1, -1))
        pos = np.empty(n, np.int64)
        pos[np.array(remaining)] = np.arange(n)
        live = np.ones(n, bool)
        spc = np.full(n, np.iinfo(np.int64).max // 4)
        path = -np.ones(n, np.int64)
        minVal = 0
        i = cur
        prev_rank = None  # per wave: columns sorted by key after the previous step
        prev_winner_wave = None
        sink = -1
        while True:
            stats["steps"] += 1
            r = minVal + C[i] - u[i] - v
            upd = live & (r < spc)
            spc = np.where(upd, r, spc)
            path = np.where(upd, i, path)
            # scipy key: (spc, assigned, assigned ? pos : -pos)
            lc = np.nonzero(live)[0]
            assigned = r4c[lc] >= 0
            key = np.lexsort((np.where(assigned, pos[lc], -pos[lc]), assigned, spc[lc]))
            order = lc[key]
            j = order[0]
            if prev_winner_wave is not None:
                wl = prev_rank[prev_winner_wave]
                # the winning wave's previous second / third best (its best won)
                ww = order[wave_of[order] == prev_winner_wave]
                if len(ww) and len(wl) > 1 and ww[0] == wl[1]:
                    stats["second_hit"] += 1
                if len(ww) and ww[0] in wl[1:3]:
                    stats["top3_hit"] += 1
                if len(ww) and upd[ww[0]]:
                    stats["improved_by_new_row"] += 1
            prev_rank = {w: order[wave_of[order] == w][:3] for w in range(NW)}
            prev_winner_wave = wave_of[j]
            minVal = spc[j]
            live[j] = False
            p = pos[j]
            last = remaining[-1]
            remaining[p] = last
            pos[last] = p
            remaining.pop()
            if r4c[j] < 0:
                sink = j
                break
            i = r4c[j]
        vis = ~live
        u[cur] += minVal
        rr = r4c[vis]
        m = rr >= 0
        u[rr[m]] += minVal - spc[vis][m]
        v[vis] -= minVal - spc[vis]
        j = sink
        while True:
            pi = path[j]
            r4c[j] = pi
            j, c4r[pi] = c4r[pi], j
            if pi == cur:
                break
        if cur % 250 == 0:
            print(cur, stats, round(time.time() - t0, 1), flush=True)
    print(stats)


if __name__ == "__main__":
    main()
