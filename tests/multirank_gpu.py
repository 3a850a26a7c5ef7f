"""Rank body of the multi-rank GPU tests (imported by the spawned ranks).

Each rank runs the product driver (santa_hip.driver.run_rounds) through the
HIP engine (GPUEngine) on cuda:0 with a gloo process group: the one-GPU box
stands in for config 4's one-process-per-GPU layout (RCCL refuses two ranks
on one device, so the exchange's all-gather goes over gloo here)."""
import os
import sys


def rank_main(rank, size, port, mode, n, rounds, seed, out):
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (os.path.join(root, "mpi-hungarian-method_amd"), here):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    from santa_hip import data as D
    from santa_hip.context import SantaGPU
    from santa_hip.driver import GPUEngine, World, run_rounds
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        torch.cuda.set_device(0)
        sd = D.synthetic(2017)
        ctx = SantaGPU.from_data(sd, 0)
        types = ctx.upload_types(sd.types)
        sums = []

        class Rec(GPUEngine):
            def score_sums(self, t):
                s = super().score_sums(t)
                sums.append(s[:2])
                return s

        res = run_rounds(Rec(ctx), types, mode=mode, n=n, seed=seed, max_rounds=rounds,
                         patience=100, world=World(rank, size, None))
        out[rank] = (types.cpu().numpy(), [(st.s_child, st.s_gift) for st in res.history],
                     [st.score for st in res.history], ctx.error_flags(), sums)
    finally:
        dist.destroy_process_group()
