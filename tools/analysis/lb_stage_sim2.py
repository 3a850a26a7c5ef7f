"""dev: staging policies of santa_lb_kernel, replayed on scipy's SAP decisions.

For one n = 2000 singles block of the bench's round 0 (lattice costs, scipy's
remaining order and tie rule), per step and per wave (NW waves of K columns
per lane, column j in wave (j // 64) // K, lane j % 64): the wave's candidate
(its minimum key) must have its row staged.  Counts, per step:
  sync      waves whose candidate's row is not staged (a dependent load),
  win_sync  steps whose WINNER's row was such a load (the next step must
            wait for it; other loads only hold the barrier),
under policy P1 (two tables per wave, stage the candidate) and P2 (+ prefetch
the best among the other lanes' minima into the other table)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mpi-hungarian-method_amd"))
from santa_hip import data as D  # noqa: E402
from santa_hip.sampler import sample_blocks, single_geometry  # noqa: E402


def main(n=2000, NW=8, K=4, block=0, max_rows=2000):
    sd = D.synthetic(2017)
    lo, count, nb = single_geometry(sd.nc, n, *sd.families)
    rows = sample_blocks(2017, 0, lo, count, 1, n, nb)[block]
    types = sd.types[rows]
    nw = sd.n_wish
    C = np.ones((n, n), dtype=np.int64)
    for i, c in enumerate(rows):
        rk = {int(g): r for r, g in enumerate(sd.wish[c])}
        a = np.array([nw - rk[t] if t in rk else 0 for t in types])
        C[i] = np.where(a > 0, -a * 256, 1)
    j_all = np.arange(n)
    wave_of = (j_all // 64) // K
    lane_of = j_all % 64
    u = np.zeros(n, np.int64)
    v = np.zeros(n, np.int64)
    r4c = -np.ones(n, np.int64)
    c4r = -np.ones(n, np.int64)
    pol = {p: {"steps": 0, "sync": 0, "win_sync": 0, "any_sync": 0, "prefetch": 0} for p in ("P1", "P2")}
    staged = {p: [[-1, -1] for _ in range(NW)] for p in pol}  # rows held by each wave's two tables
    for cur in range(min(n, max_rows)):
        remaining = list(range(n - 1, -1, -1))
        pos = np.empty(n, np.int64)
        pos[np.array(remaining)] = np.arange(n)
        live = np.ones(n, bool)
        spc = np.full(n, np.iinfo(np.int64).max // 4)
        path = -np.ones(n, np.int64)
        minVal = 0
        i = cur
        while True:
            r = minVal + C[i] - u[i] - v
            upd = live & (r < spc)
            spc = np.where(upd, r, spc)
            path = np.where(upd, i, path)
            assigned = r4c >= 0
            tie = np.where(assigned, 2048 + pos, 2047 - pos)
            key = np.where(live, spc * 4096 + tie, np.iinfo(np.int64).max)
            j = int(np.argmin(key))
            for p in pol:
                st = pol[p]
                st["steps"] += 1
                nsync = 0
                win_sync = False
                for w in range(NW):
                    m = wave_of == w
                    kw = np.where(m, key, np.iinfo(np.int64).max)
                    b = int(np.argmin(kw))
                    if kw[b] == np.iinfo(np.int64).max:
                        continue
                    if r4c[b] >= 0:
                        row = int(r4c[b])
                        tb = staged[p][w]
                        if row not in tb:
                            nsync += 1
                            # the table not holding the other staged row... replace the older one
                            tb[0], tb[1] = tb[1], row
                            if b == j:
                                win_sync = True
                        if p == "P2":
                            kw2 = np.where(m & (lane_of != lane_of[b]), key, np.iinfo(np.int64).max)
                            b2 = int(np.argmin(kw2))
                            if kw2[b2] != np.iinfo(np.int64).max and r4c[b2] >= 0:
                                row2 = int(r4c[b2])
                                if row2 not in tb:
                                    st["prefetch"] += 1
                                    # keep the candidate's row, the other table gets the prefetch
                                    keep = row
                                    staged[p][w] = [keep, row2]
                st["sync"] += nsync
                st["any_sync"] += nsync > 0
                st["win_sync"] += win_sync
            minVal = spc[j]
            live[j] = False
            pp = pos[j]
            last = remaining[-1]
            remaining[pp] = last
            pos[last] = pp
            remaining.pop()
            if r4c[j] < 0:
                sink = j
                break
            i = r4c[j]
        vis = ~live
        u[cur] += minVal
        rr = r4c[vis]
        mm = rr >= 0
        u[rr[mm]] += minVal - spc[vis][mm]
        v[vis] -= minVal - spc[vis]
        jj = sink
        while True:
            pi = path[jj]
            r4c[jj] = pi
            jj, c4r[pi] = c4r[pi], jj
            if pi == cur:
                break
        if cur % 250 == 0:
            print(cur, pol, flush=True)
    for p, st in pol.items():
        s = st["steps"]
        print(p, {k: (round(x / s, 3) if k != "steps" else x) for k, x in st.items()})


if __name__ == "__main__":
    main()
