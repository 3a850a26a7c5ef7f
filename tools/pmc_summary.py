"""dev: per-wave-step SQ counters of the block kernel from tools/pmc_probe.sh output"""
import csv, json, collections, sys
d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in ("sq1", "sq2"):
    for r in csv.DictReader(open(f"{d}/{f}_counter_collection.csv")):
        if "santa" in r["Kernel_Name"]:
            agg[r["Kernel_Name"][:45]][r["Counter_Name"]] += float(r["Counter_Value"])
pr = json.loads(open(f"{d}/probe_sq1.json").read().strip().splitlines()[-1])
for k, v in agg.items():
    w = v["SQ_WAVES"]
    per = pr["steps_total"] * (w / pr["blocks"])
    print(k, "waves", w, "steps", pr["steps_total"])
    for c, x in sorted(v.items()):
        if c != "SQ_WAVES":
            print(f"  {c:26s} per wave-step {x / per:9.2f}")
