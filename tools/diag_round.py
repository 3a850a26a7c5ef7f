"""dev: one full singles round (3730 blocks, the default design) against the
CPU oracle, block by block: col, cost, the new types and the delta sums.
Prints one JSON line.  SANTA_HIP_LIB selects the library (A/B of builds).
  python tools/diag_round.py [--seed 8] [--round 0] [--blocks 0] [--flags 0]"""
import argparse
import concurrent.futures as cf
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-hungarian-method_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch  # noqa: E402

import oracle  # noqa: E402  (dev tool: the checker)
from santa_hip import data as D  # noqa: E402
from santa_hip.context import SantaGPU  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=8)
    ap.add_argument("--round", type=int, default=0)
    ap.add_argument("--blocks", type=int, default=0)
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--n", type=int, default=256)
    a = ap.parse_args()
    sd = D.synthetic(2017)
    ctx = SantaGPU.from_data(sd, 0)
    _, _, _, nb = ctx.geometry(a.mode, a.n)
    B = a.blocks or nb
    n = a.n
    rows = ctx.sample_blocks(a.mode, n, B, a.seed, a.round)
    types = ctx.upload_types(sd.types)
    col = torch.empty(B * n, dtype=torch.int32, device="cuda")
    cost = torch.empty(B, dtype=torch.int64, device="cuda")
    steps = torch.empty(B, dtype=torch.int64, device="cuda")
    delta = torch.zeros(2, dtype=torch.int64, device="cuda")
    ctx.solve_blocks(a.mode, rows, n, types, col=col, cost=cost, steps=steps, delta=delta, flags=a.flags)
    torch.cuda.synchronize()
    r = rows.cpu().numpy().reshape(B, n)
    gcol, gcost, gst = col.cpu().numpy().reshape(B, n), cost.cpu().numpy(), steps.cpu().numpy()
    t_host = sd.types.copy()
    res = {}

    def work(b0):
        c, k = oracle.round_blocks(a.mode, sd.wish, t_host, r[b0:b0 + 64], ng=sd.ng)
        return b0, c, k
    bad_col, bad_cost = [], []
    with cf.ThreadPoolExecutor(16) as ex:
        for b0, c, k in ex.map(work, range(0, B, 64)):
            for j in range(len(k)):
                if not np.array_equal(c[j], gcol[b0 + j]):
                    bad_col.append(b0 + j)
                if k[j] != gcost[b0 + j]:
                    bad_cost.append(b0 + j)
    gt = types.cpu().numpy()
    s0 = oracle.score_sums(sd.wish, sd.goodkids, sd.types)
    s1 = oracle.score_sums(sd.wish, sd.goodkids, t_host)
    sg = oracle.score_sums(sd.wish, sd.goodkids, gt)
    res.update(B=B, bad_col=len(bad_col), bad_cost=len(bad_cost), first_bad_col=bad_col[:8],
               first_bad_cost=bad_cost[:8], types_equal=bool(np.array_equal(gt, t_host)),
               types_diff=int((gt != t_host).sum()), delta=delta.cpu().tolist(),
               oracle_delta=[s1[0] - s0[0], s1[1] - s0[1]], gpu_state_delta=[sg[0] - s0[0], sg[1] - s0[1]],
               err=ctx.error_flags(), lib=os.environ.get("SANTA_HIP_LIB", "default"))
    wrong = np.nonzero(gt != t_host)[0]
    if wrong.size:
        pos = {int(c): (b, i) for b in range(B) for i, c in enumerate(r[b])} if wrong.size else {}
        res["wrong"] = [{"child": int(c), "block": pos.get(int(c), (-1, -1))[0], "i": pos.get(int(c), (-1, -1))[1],
                         "gpu": int(gt[c]), "oracle": int(t_host[c]), "start": int(sd.types[c])}
                        for c in wrong[:80]]
    if bad_cost:
        b = bad_cost[0]
        res["example"] = {"block": b, "gpu_cost": int(gcost[b]), "steps": int(gst[b])}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
