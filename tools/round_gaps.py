"""dev: the time between two rounds' block kernels in a rocprofv3 kernel trace
of bench.py (--kernel-trace --output-format csv), and what runs in between.

    python tools/round_gaps.py <kernel_trace.csv> [main-kernel-substring] [label]

Prints one JSON object: rounds, median/min/max gap (end of one round's main
kernel to the start of the next; gaps > 200 us, outside the round loop,
dropped) and the kernels of one median gap (name, stream, duration in us)."""
import csv
import json
import re
import statistics
import sys


def short(name: str) -> str:
    name = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "")
    return name.split("(")[0][:48]


def main():
    path = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else "santa_sp3_kernel"
    label = sys.argv[3] if len(sys.argv) > 3 else path
    rows = list(csv.DictReader(open(path)))
    name_k = next(k for k in rows[0] if k.lower() in ("kernel_name", "name"))
    s_k = next(k for k in rows[0] if k.lower().startswith("start_timestamp"))
    e_k = next(k for k in rows[0] if k.lower().startswith("end_timestamp"))
    st_k = next((k for k in rows[0] if k.lower() in ("stream_id", "queue_id")), None)
    ev = sorted(((int(r[s_k]), int(r[e_k]), r[name_k], r.get(st_k, "?") if st_k else "?") for r in rows))
    mains = [e for e in ev if key in e[2]]
    gaps = []
    for a, b in zip(mains, mains[1:]):
        g = (b[0] - a[1]) / 1e3
        if 0 <= g <= 200:
            between = [(short(x[2]), x[3], round((x[1] - x[0]) / 1e3, 1)) for x in ev
                       if x[0] >= a[1] and x[1] <= b[0]]
            gaps.append((g, between))
    gaps.sort(key=lambda t: t[0])
    med = gaps[len(gaps) // 2] if gaps else (None, [])
    print(json.dumps({label: {"rounds": len(gaps), "median_gap_us": round(statistics.median(g for g, _ in gaps), 1)
                              if gaps else None,
                              "min_gap_us": round(gaps[0][0], 1) if gaps else None,
                              "max_gap_us": round(gaps[-1][0], 1) if gaps else None,
                              "kernels_between_example": med[1]}}))


if __name__ == "__main__":
    main()
