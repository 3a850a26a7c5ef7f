#!/bin/bash
# round-5 GPU session 3: santa_lb_kernel segment profile (lone n = 2000 block,
# full round 0 and round 10)
cd /root/repo
timeout -k 10 120 python tools/probe.py --n 2000 --blocks 1 --phase solve --reps 2 --lb-segments > gpurun_out/r5c_lone.json || exit 1
timeout -k 10 200 python tools/probe.py --n 2000 --phase solve --reps 1 --lb-segments > gpurun_out/r5c_round0.json || exit 1
timeout -k 10 200 python tools/probe.py --n 2000 --phase solve --reps 1 --lb-segments --state-round 10 > gpurun_out/r5c_round10.json || exit 1
python - <<'PY'
import json
for f in ("r5c_lone", "r5c_round0", "r5c_round10"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, d["solve"]["ms"], d["steps_max"])
    for k, v in d["lb_segments_cycles_per_step_maxblock"].items():
        print("  ", k, v)
    print("   staged", d["lb_staged_per_step_maxblock"])
    print("   prefetched", d.get("lb_prefetched_per_step_maxblock"))
    print("   sync load cycles", d.get("lb_sync_load_cycles_maxblock"))
    print("   mean", d["lb_segments_mean_over_waves_all_blocks"])
PY
echo all-done
