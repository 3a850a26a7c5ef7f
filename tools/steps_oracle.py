"""Dev (CPU only): per-block Dijkstra step counts of successive full singles
rounds from the synthetic baseline, computed with the CPU oracle (test
infrastructure, used here as a study tool), for the round-schedule model in
tools/sched_model.py.  Writes gpurun_out/steps_oracle_<R>.npz: rows<r> [B, n],
steps<r> [B]."""
import argparse
import concurrent.futures as cf
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-hungarian-method_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402
from santa_hip import data as D  # noqa: E402
from santa_hip.sampler import sample_blocks, single_geometry  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=20)
ap.add_argument("--seed", type=int, default=2017)
ap.add_argument("--threads", type=int, default=8)
args = ap.parse_args()

sd = D.synthetic(args.seed)
tri, tw = sd.families
lo, count, nb = single_geometry(sd.nc, 256, tri, tw)
t = sd.types.copy()
out = {}


def one(blk):
    st = np.zeros(2, dtype=np.uint64)
    oracle.round_blocks(0, sd.wish, t, blk[None, :], stats=st, ng=sd.ng)
    return int(st[0])


with cf.ThreadPoolExecutor(args.threads) as ex:
    for r in range(args.rounds):
        rows = sample_blocks(args.seed, r, lo, count, 1, 256, nb)
        steps = np.array(list(ex.map(one, rows)), dtype=np.int64)
        out[f"rows{r}"] = rows
        out[f"steps{r}"] = steps
        print(r, steps.mean(), steps.max(), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"steps_oracle_{args.rounds}.npz"), **out)
