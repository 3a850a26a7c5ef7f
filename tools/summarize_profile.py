"""Turn a tools/profile_round.sh output directory into profiles/<tag>_*.

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, verbatim) and
profiles/<tag>_summary.json: per-kernel average duration from the trace,
HBM bytes per launch from FETCH_SIZE / WRITE_SIZE (KB, x1024), and the SQ
counters per wave and per Dijkstra step of the block kernel."""
import csv
import glob
import hashlib
import json
import os
import shutil
import sys
from collections import defaultdict


def pmc(path):
    agg = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(path):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
    return agg


def by_short(agg, main=None):
    """Merge the instantiations of one kernel (e.g. santa_vt_kernel<0, true>
    and its fallback launch santa_vt_kernel<0, false>) under the short name:
    counters summed (HBM bytes of the whole solve), or, with `main`, the
    instantiation with the largest `main` counter kept (the launch that did
    the work, for per-wave and occupancy figures)."""
    out = {}
    for k, v in agg.items():
        s = short(k)
        if s not in out:
            out[s] = dict(v)
        elif main is None:
            for c, x in v.items():
                out[s][c] = out[s].get(c, 0.0) + x
        elif v.get(main, 0.0) > out[s].get(main, 0.0):
            out[s] = dict(v)
    return out


def short(name):
    for key in ("santa_sp3_kernel", "santa_dt_kernel", "santa_sp2_kernel", "santa_tile_kernel", "santa_sp_kernel", "santa_vt_kernel", "santa_sw_kernel", "santa_block_kernel",
                "santa_lb_kernel", "santa_big_kernel", "score_kernel", "publish_kernel",
                "sample_kernel", "lsap_i64_kernel", "lsap_f64_kernel"):
        if key in name:
            return key
    return name[:60]


def main(src, tag, root):
    prof = os.path.join(root, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace_kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{tag}_kernel_stats.csv"))
    for part in ("fetch", "write", "sq1", "sq2", "occ", "fetch_score"):
        f = os.path.join(src, f"{part}_counter_collection.csv")
        if os.path.exists(f):
            shutil.copy(f, os.path.join(prof, f"{tag}_pmc_{part}.csv"))
    trace = defaultdict(list)
    for f in glob.glob(os.path.join(src, "trace_kernel_trace.csv")):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
        for r in rows:
            trace[short(r["Kernel_Name"])].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    ksrc = os.path.join(root, "mpi-hungarian-method_amd", "csrc", "santa_hip.hip")
    out = {"tag": tag, "source_sha16": hashlib.sha256(open(ksrc, "rb").read()).hexdigest()[:16],
           "trace_ms": {k: {"calls": len(v), "avg_ms": sum(v) / len(v),
                                         "min_ms": min(v), "max_ms": max(v)}
                                     for k, v in trace.items()}}
    # the bench's timed rounds: launches [warmup, warmup + steps) of the block
    # kernel (bench.py runs `warmup` untimed rounds first, one extra launch after)
    bj = os.path.join(src, "bench_under_trace.json")
    if os.path.exists(bj):
        b = json.loads(open(bj).read().strip().splitlines()[-1])
        w, k = b["warmup"], b["steps"]
        kn = b["roofline"]["kernel"].split(" ")[0].split("<")[0]
        # the register-tile sparse design runs two kernels per solve launch
        # (one since round 4 with the packed wishlists: the tile is built in-kernel)
        kns = ["santa_tile_kernel", kn] if kn in ("santa_sp2_kernel", "santa_sp3_kernel") else [kn]
        kns = [x for x in kns if x in trace]
        vs = [trace.get(x, []) for x in kns]
        if all(len(v) >= w + k for v in vs):
            t = [sum(v[i] for v in vs) for i in range(w, w + k)]
            out["timed_window"] = {"kernels": kns, "launches": f"[{w}, {w + k})",
                                   "avg_ms": sum(t) / len(t),
                                   "bench_kernel_avg_ms": b["roofline"]["kernel_avg_ms"]}
            rs = b["roofline"].get("kernel_avg_rounds")
            if rs:  # the rounds the bench's events bracketed: the same launches in the trace
                ts = [t[r] for r in rs if r < len(t)]
                out["timed_window"]["event_rounds"] = rs
                out["timed_window"]["event_rounds_avg_ms"] = sum(ts) / len(ts)
    fetch = pmc(os.path.join(src, "fetch_counter_collection.csv"))
    write = pmc(os.path.join(src, "write_counter_collection.csv"))
    fscore = pmc(os.path.join(src, "fetch_score_counter_collection.csv"))
    hbm = {}
    for d, key in ((fetch, "FETCH_SIZE"), (write, "WRITE_SIZE"), (fscore, "FETCH_SIZE")):
        for k, v in by_short(d).items():
            hbm.setdefault(k, {})[key + "_bytes"] = v.get(key, 0.0) * 1024
    out["hbm_bytes_per_launch"] = hbm
    probe = {}
    pj = os.path.join(src, "probe_sq1.json")
    if os.path.exists(pj):
        probe = json.loads(open(pj).read().strip().splitlines()[-1])
    sq = pmc(os.path.join(src, "sq1_counter_collection.csv"))
    for k, v in pmc(os.path.join(src, "sq2_counter_collection.csv")).items():
        sq[k].update(v)
    steps = probe.get("steps_total")
    sqs = {}
    for k, v in by_short(sq, "SQ_WAVE_CYCLES").items():
        waves = v.get("SQ_WAVES", 0) or 1
        e = {c: x for c, x in v.items()}
        if steps:
            wps = steps * waves / probe["blocks"]
            e["per_wave_step_quadcycles"] = {c: x / wps for c, x in v.items() if c.startswith("SQ_")
                                             and c != "SQ_WAVES"}
        sqs[k] = e
    out["sq"] = sqs
    out["probe"] = probe
    # occupancy and LDS activity (own PMC pass, tools/profile_round.sh "occ"):
    #   mean resident waves per SIMD over the launch = SQ_WAVE_CYCLES (quad-
    #   cycles, x4) / (GRBM_GUI_ACTIVE / 8 XCDs) / (CUs x 4 SIMDs), the
    #   OccupancyPercent formula of rocprofv3's derived counters;
    #   LDS-array busy = SQ_LDS_IDX_ACTIVE / (GRBM_GUI_ACTIVE / 8 x CUs);
    #   conflict share = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.
    n_cu = 256
    occ = {}
    for k, v in by_short(pmc(os.path.join(src, "occ_counter_collection.csv")), "GRBM_GUI_ACTIVE").items():
        grbm = v.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        if not grbm:
            continue
        e = {"kernel_cycles_per_xcd": grbm,
             "mean_waves_per_simd": 4.0 * v.get("SQ_WAVE_CYCLES", 0.0) / grbm / (n_cu * 4)}
        if v.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_array_busy_frac"] = v["SQ_LDS_IDX_ACTIVE"] / (grbm * n_cu)
            e["lds_bank_conflict_frac"] = v.get("SQ_LDS_BANK_CONFLICT", 0.0) / v["SQ_LDS_IDX_ACTIVE"]
            e["lds_insts"] = v.get("SQ_INSTS_LDS", 0.0)
        occ[k] = e
    if occ:
        out["occupancy_lds"] = occ
    po = os.path.join(src, "probe_occ.json")
    if os.path.exists(po):
        out["probe_occ"] = json.loads(open(po).read().strip().splitlines()[-1])
    json.dump(out, open(os.path.join(prof, f"{tag}_summary.json"), "w"), indent=1)
    print(json.dumps(out["trace_ms"], indent=1))
    print(json.dumps(hbm, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
