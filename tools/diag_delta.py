import sys, numpy as np, torch
sys.path.insert(0, "mpi-hungarian-method_amd"); sys.path.insert(0, "oracle")
import oracle
from santa_hip import data as D
from santa_hip.context import SantaGPU
sd = D.synthetic(2017)
ctx = SantaGPU.from_data(sd, 0)
mode, n = 0, 256
_, _, _, nb = ctx.geometry(mode, n)
rows = ctx.sample_blocks(mode, n, nb, 9, 0)
r = rows.cpu().numpy().reshape(nb, n)
wish = sd.wish
def happy(child, t):
    w = wish[child]
    idx = np.nonzero(w == t)[0]
    return 2 * (100 - idx[0]) if idx.size else -1
bad = 0
for b in range(nb):
    types = ctx.upload_types(sd.types)
    delta = torch.zeros(2, dtype=torch.int64, device="cuda")
    col = torch.empty(n, dtype=torch.int32, device="cuda")
    ctx.solve_blocks(mode, rows[b*n:(b+1)*n], n, types, col=col, delta=delta)
    c = col.cpu().numpy()
    blk = r[b]
    old = sd.types[blk]; new = old[c]
    dch = sum(happy(ch, tn) - happy(ch, to) for ch, to, tn in zip(blk, old, new))
    g = delta.cpu().tolist()[0]
    if g != dch:
        bad += 1
        print("block", b, "gpu", g, "cpu", dch)
        for i, ch in enumerate(blk):
            pass
        if bad > 3: break
print("bad", bad, "fallback flags", ctx.error_flags())
