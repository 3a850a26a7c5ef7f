"""Where a block's Dijkstra steps fall (dev analysis, CPU only): per-cur step
counts of scipy's SAP on the round-0 singles blocks of the seeded synthetic
instance, and how well the steps of the first c rows predict a block's total
(the question behind an LPT order or priority for the longest blocks).

    python tools/steps_by_cur.py [n_blocks]
"""
import ctypes
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-hungarian-method_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    import oracle
    from santa_hip import data as D, sampler
    from santa_hip.sampler import single_geometry
    so = "/tmp/steps_by_cur.so"
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", so,
                    os.path.join(ROOT, "tools", "calib", "steps_by_cur.c")], check=True)
    L = ctypes.CDLL(so)
    sd = D.synthetic(2017)
    tri, tw = sampler.family_sizes(sd.nc)
    lo, count, nb = single_geometry(sd.nc, 256, tri, tw)
    rows = sampler.sample_blocks(2017, 0, lo, count, 1, 256, nb)
    NB = int(sys.argv[1]) if len(sys.argv) > 1 else 800
    out = np.zeros((NB, 256), np.int32)

    def one(b):
        C = np.ascontiguousarray(oracle.cost_single(sd.wish, sd.types, rows[b]), dtype=np.int64)
        L.steps_by_cur(256, C.ctypes.data_as(ctypes.c_void_p), out[b].ctypes.data_as(ctypes.c_void_p))

    with ThreadPoolExecutor(8) as ex:
        list(ex.map(one, range(NB)))
    tot = out.sum(1)
    print(f"blocks {NB}: steps mean {tot.mean():.0f} max {tot.max()}")
    cum = out.cumsum(1)
    top = np.argsort(-tot)[:8]
    for c in (32, 64, 128, 192, 224):
        r = np.corrcoef(cum[:, c - 1], tot)[0, 1]
        print(f"first {c} rows: corr(prefix, total) = {r:.3f}; top-8 blocks have "
              f"{cum[top, c - 1].mean() / tot[top].mean():.1%} of their steps done")


if __name__ == "__main__":
    main()
