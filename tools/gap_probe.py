"""Where the time between two rounds' block kernels goes (host-side A/B, one
process): the same rounds 0..R-1 from the baseline state, enqueued as
  bare     : pre-sampled rows, solve only, no host sync (the kernel floor)
  d_main   : + delta zeroed and copied to the host on the round's stream
  d_side   : + delta copied / zeroed on a side stream after a ready event
  sync     : d_side with the host waiting on round r - 1 after enqueuing round r
  loop_pK_side / _main: santa_hip.driver.run_rounds(pipeline=True), the
             bench's loop, sampling K rounds ahead (0: on the round's stream),
             the bookkeeping after the snapshot on the side / round's stream
  sync_sample_side / _main: sync with a sampling kernel per round on the side
             stream (concurrent with the solve) / on the round's stream
and prints one JSON line of ms per round for each.
    python tools/gap_probe.py [--rounds 60] [--mode single|twins]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-hungarian-method_amd"))

import torch  # noqa: E402

from santa_hip import data as D  # noqa: E402
from santa_hip.context import SantaGPU  # noqa: E402
from santa_hip.driver import GPUEngine, World, run_rounds  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=60)
    ap.add_argument("--mode", default="single")
    ap.add_argument("--seed", type=int, default=2017)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--only", default="", help="comma-separated variant names")
    args = ap.parse_args()
    mode = {"single": 0, "twins": 1}[args.mode]
    n, R = 256, args.rounds
    sd = D.synthetic(args.seed)
    ctx = SantaGPU.from_data(sd, 0)
    _, _, _, nb = ctx.geometry(mode, n)
    rows = [ctx.sample_blocks(mode, n, nb, args.seed, r) for r in range(R)]
    types = ctx.upload_types(sd.types)
    base = types.clone()
    snap = torch.empty_like(types)
    dl = [torch.zeros(2, dtype=torch.int64, device="cuda") for _ in range(2)]
    dh = [torch.zeros(2, dtype=torch.int64).pin_memory() for _ in range(2)]
    side = torch.cuda.Stream()
    scratch = [torch.empty(nb * n, dtype=torch.int32, device="cuda") for _ in range(3)]
    main_s = torch.cuda.current_stream()

    def run(variant, side_sample=False, main_sample=False):
        types.copy_(base)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        zev = [None, None]
        prev = None
        for r in range(R):
            k = r & 1
            d = dl[k] if variant != "bare" and variant != "snap" else None
            if variant in ("d_side", "sync") and zev[k] is not None:
                if not zev[k].query():
                    main_s.wait_event(zev[k])
            if variant == "d_main":
                d.zero_()
            if main_sample:
                ctx.sample_blocks(mode, n, nb, args.seed, r, out=scratch[0])
            ctx.solve_blocks(mode, rows[r], n, types, delta=d)
            if side_sample:
                fr = torch.cuda.Event()
                fr.record(main_s)
                with torch.cuda.stream(side):
                    side.wait_event(fr)
                    ctx.sample_blocks(mode, n, nb, args.seed, r + 2, out=scratch[r % 3])
            if variant != "bare":
                snap.copy_(types)
            if variant == "d_main":
                dh[k].copy_(d, non_blocking=True)
            if variant in ("d_side", "sync"):
                ready = torch.cuda.Event()
                ready.record(main_s)
                with torch.cuda.stream(side):
                    side.wait_event(ready)
                    dh[k].copy_(d, non_blocking=True)
                    done = torch.cuda.Event()
                    done.record(side)
                    d.zero_()
                    z = torch.cuda.Event()
                    z.record(side)
                zev[k] = z
                if variant == "sync":
                    if prev is not None:
                        prev.synchronize()
                    prev = done
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / R

    def loop(prefetch=GPUEngine.PREFETCH, side=True, mailbox=True, fused=True):
        types.copy_(base)

        class Eng(GPUEngine):
            PREFETCH = prefetch
            SIDE_STREAM = side
            MAILBOX = mailbox
            FUSED_SAMPLING = fused
        eng = Eng(ctx)
        s = ctx.score_sums(types)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run_rounds(eng, types, mode=mode, n=n, seed=args.seed, max_rounds=R, patience=1 << 30,
                   world=World(), sums0=(s[0], s[1]), pipeline=True)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / R

    out = {}
    variants = {"bare": lambda: run("bare"), "d_main": lambda: run("d_main"), "sync": lambda: run("sync"),
                "sync_sample_side": lambda: run("sync", side_sample=True),
                "sync_sample_main": lambda: run("sync", main_sample=True),
                "loop_p2_side": lambda: loop(2, True), "loop_p0_main": lambda: loop(0, False),
                "loop_p0_side": lambda: loop(0, True), "loop_p2_main": lambda: loop(2, False),
                "loop_p1_side": lambda: loop(1, True),
                "loop_r5": lambda: loop(0, True, True, True), "loop_r5_nomail": lambda: loop(0, True, False, True),
                "loop_r5_nofuse": lambda: loop(0, True, True, False),
                "loop_r5_neither": lambda: loop(0, True, False, False)}
    if args.only:
        variants = {k: v for k, v in variants.items() if k in args.only.split(",")}
    for rep in range(args.reps + 1):
        for name, f in variants.items():
            v = round(f(), 4)
            if rep:  # (rep 0 warms every path up)
                out.setdefault(name, []).append(v)
    out = {k: sorted(v) for k, v in out.items()}
    med = {k: v[len(v) // 2] for k, v in out.items()}
    print(json.dumps({"mode": args.mode, "rounds": R, "median_ms_per_round": med, "ms_per_round": out}))


if __name__ == "__main__":
    main()
