"""dev: time lsap_solve_batched_hash for a few (n, B) on the library SANTA_HIP_LIB selects (A/B).
    python tools/lsap_time.py [NxB ...]     (default: 256x512 512x256 1024x256 256x4096)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-hungarian-method_amd"))
import torch  # noqa: E402
import santa_hip  # noqa: E402

cases = [tuple(int(x) for x in c.split("x")) for c in sys.argv[1:]] or [(256, 512), (512, 256), (1024, 256),
                                                                         (256, 4096)]
for n, B in cases:
    santa_hip.solve_hash(7, 1 << 16, n, B)
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        santa_hip.solve_hash(7, 1 << 16, n, B)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    print(json.dumps({"n": n, "B": B, "ms": min(ts)}))
