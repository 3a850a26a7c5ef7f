"""Kernel probe: times the fused block kernel's phases on round 0 of the
benchmark workload (build only vs build+solve), with HIP events.  Used with
rocprofv3 --pmc to attribute per-step cycles.  Not part of the product."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-hungarian-method_amd"))
import torch  # noqa: E402

from santa_hip import _lib, data as D  # noqa: E402
from santa_hip.context import SantaGPU  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--blocks", type=int, default=0, help="0 = full round")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--phase", choices=["all", "build", "solve", "score"], default="all")
    ap.add_argument("--flags", type=int, default=0, help="extra SH_FLAG_* bits (8 = LDS tile)")
    ap.add_argument("--budget", type=int, default=0, help="sparse kernel LDS bytes per block (0 = default)")
    ap.add_argument("--timing", action="store_true", help="per-phase in-kernel timing (sparse kernel)")
    ap.add_argument("--segments", action="store_true",
                    help="santa_sp3_kernel (santa_dt_kernel with --flags 4096): shader cycles per Dijkstra step "
                         "by segment (A fetch+scatter+LDS, B relax+argmin, C decode+book-keeping, "
                         "D per-Dijkstra work per step)")
    ap.add_argument("--lb-segments", action="store_true",
                    help="santa_lb_kernel (n > 256 singles): cycles per step by segment, per wave "
                         "(0 relax, 1 wave min, 2 candidate + staging + fold, 3 barrier, 4 decode, "
                         "5 per-Dijkstra) and rows staged per step")
    ap.add_argument("--state-round", type=int, default=0,
                    help="time round R of the optimisation: first apply rounds 0..R-1 (default kernel)")
    a = ap.parse_args()
    sd = D.synthetic(2017)
    ctx = SantaGPU.from_data(sd, 0)
    cap = ctx.set_sparse_budget(a.budget)
    _, _, _, nb = ctx.geometry(a.mode, a.n)
    B = a.blocks or nb
    base = ctx.upload_types(sd.types)
    for r in range(a.state_round):
        ctx.solve_blocks(a.mode, ctx.sample_blocks(a.mode, a.n, nb, 2017, r), a.n, base)
    rows = ctx.sample_blocks(a.mode, a.n, B, 2017, a.state_round)
    steps = torch.empty(B, dtype=torch.int64, device="cuda")
    out = {}
    for name, fl in (("build", _lib.SH_FLAG_BUILD_ONLY), ("solve", 0)):
        if a.phase not in ("all", name):
            continue
        ts = []
        for _ in range(a.reps):
            t = base.clone()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ctx.solve_blocks(a.mode, rows, a.n, t, steps=steps, flags=fl | a.flags)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        out[name] = {"ms": min(ts), "all_ms": ts}
    if a.phase in ("all", "score"):
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ctx.score_sums_async(base)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        out["score"] = {"ms": min(ts), "all_ms": ts}
    if a.timing:  # dev: per-phase wall-clock ticks of the sparse kernel (100 MHz)
        t = base.clone()
        col = torch.zeros(B * a.n, dtype=torch.int32, device="cuda")
        ctx.solve_blocks(a.mode, rows, a.n, t, steps=steps, col=col, flags=_lib.SH_FLAG_TIMING | a.flags)
        cv = col.view(B, a.n).cpu().numpy().astype(float)
        out["colsort_us"] = float(cv[:, 0].mean()) / 100.0
        solve_cycles = cv[:, 1]
        v = steps.cpu().numpy().astype("uint64")
        ph = [(v & 0x1FFFFF), (v >> 21) & 0x1FFFFF, (v >> 42) & 0x1FFFFF]
        built, solved, done = [x.astype(float) / 100.0 for x in ph]  # us
        out["timing_us"] = {"build_mean": built.mean(), "build_max": built.max(),
                            "solve_mean": (solved - built).mean(), "solve_max": (solved - built).max(),
                            "epilogue_mean": (done - solved).mean(), "total_max": done.max()}
        steps.zero_()
        ctx.solve_blocks(a.mode, rows, a.n, base.clone(), steps=steps, flags=a.flags)
        sv = steps.cpu().numpy().astype(float)
        wall_us = (solved - built)
        out["timing_us"]["shader_MHz"] = float(solve_cycles.sum() / wall_us.sum())
        out["timing_us"]["cycles_per_step"] = float(solve_cycles.sum() / sv.sum())
        imax = int(sv.argmax())
        out["timing_us"]["cycles_per_step_maxblock"] = float(solve_cycles[imax] / sv[imax])
    if a.segments:
        t = base.clone()
        col = torch.zeros(B * a.n, dtype=torch.int32, device="cuda")
        ctx.solve_blocks(a.mode, rows, a.n, t, steps=steps, col=col, flags=_lib.SH_FLAG_TIMING | a.flags)
        cv = col.view(B, a.n)[:, :7].cpu().numpy().astype(float)
        sv = steps.cpu().numpy().astype(float)
        imax = int(sv.argmax())
        names = ["A_fetch_scatter_lds", "B_relax_argmin", "C_decode_bookkeeping", "D_per_dijkstra"]
        if a.flags & 4096:  # (santa_dt_kernel, forced by SH_FLAG_DT_TILE)
            names = ["A_lds_group", "B_relax_argmin", "C_decode", "D_per_dijkstra"]
        elif a.mode == 1:  # (the 4-wave twins kernel, sap_solve_mw_sc: wave 0's segments)
            names = ["A_dual_row_loads", "B_relax_rowmin_fold", "C_barrier", "D_word_decode", "E_per_dijkstra"]
        elif (a.flags & 8) == 0:  # (santa_sp3_kernel: A split at the LDS issue, A1 = tile fetch + fields)
            names = ["A2_lds_bookkeeping", "B_relax_argmin", "C_decode", "D0_setup", "A1_tile_fetch",
                     "D1_dual_update", "D2_augment"]
        cv = cv[:, :len(names)]
        out["segments_cycles_per_step"] = {nm: float(cv[:, q].sum() / sv.sum()) for q, nm in enumerate(names)}
        out["segments_cycles_per_step_maxblock"] = {nm: float(cv[imax, q] / sv[imax])
                                                    for q, nm in enumerate(names)}
    if a.lb_segments:
        t = base.clone()
        col = torch.zeros(B * a.n, dtype=torch.int32, device="cuda")
        ctx.solve_blocks(a.mode, rows, a.n, t, steps=steps, col=col, flags=_lib.SH_FLAG_TIMING | a.flags)
        cfull = col.view(B, a.n).cpu().numpy().astype(float)
        cv = cfull[:, :128].reshape(B, 16, 8)
        lat = cfull[:, 128:144]
        sv = steps.cpu().numpy().astype(float)
        nwv = int((cv[0, :, 0] > 0).sum())
        names = ["relax", "wave_min", "candidate_stage_fold", "barrier", "decode_bookkeeping", "per_dijkstra"]
        imax = int(sv.argmax())
        out["lb_waves"] = nwv
        out["lb_segments_cycles_per_step_maxblock"] = {
            nm: [round(float(cv[imax, w, q] / sv[imax]), 1) for w in range(nwv)] for q, nm in enumerate(names)}
        out["lb_staged_per_step_maxblock"] = [round(float(cv[imax, w, 6] / sv[imax]), 3) for w in range(nwv)]
        out["lb_prefetched_per_step_maxblock"] = [round(float(cv[imax, w, 7] / sv[imax]), 3) for w in range(nwv)]
        out["lb_sync_load_cycles_maxblock"] = [round(float(lat[imax, w] / max(cv[imax, w, 6], 1)), 1)
                                               for w in range(nwv)]
        out["lb_segments_mean_over_waves_all_blocks"] = {
            nm: round(float(cv[:, :nwv, q].sum() / nwv / sv.sum()), 1) for q, nm in enumerate(names)}
    out["blocks"] = B
    out["n"] = a.n
    out["mode"] = a.mode
    out["budget"] = a.budget
    out["cap"] = cap
    out["flags"] = a.flags
    out["state_round"] = a.state_round
    out["steps_total"] = int(steps.sum())
    out["steps_per_block"] = int(steps.sum()) / B
    out["steps_max"] = int(steps.max())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
