"""Dev: per-block Dijkstra step counts of full singles rounds (for studying the
kernel's tail / block-order heuristics offline).  Saves rows, steps and the
types before each saved round to gpurun_out/steps_dump.npz."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-hungarian-method_amd"))
import torch  # noqa: E402

from santa_hip import data as D  # noqa: E402
from santa_hip.context import SantaGPU  # noqa: E402

sd = D.synthetic(2017)
ctx = SantaGPU.from_data(sd, 0)
_, _, _, nb = ctx.geometry(0, 256)
t = ctx.upload_types(sd.types)
out = {}
save = {0, 1, 5, 10, 19}
for r in range(20):
    rows = ctx.sample_blocks(0, 256, nb, 2017, r)
    steps = torch.zeros(nb, dtype=torch.int64, device="cuda")
    if r in save:
        out[f"types{r}"] = t.cpu().numpy()
    ctx.solve_blocks(0, rows, 256, t, steps=steps)
    if r in save:
        out[f"rows{r}"] = rows.cpu().numpy()
        out[f"steps{r}"] = steps.cpu().numpy()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "steps_dump.npz"), **out)
print("saved", {k: v.shape for k, v in out.items()})
