#!/bin/bash
# round-4 GPU session 15: the delta all-reduce waited by the side stream
# (driver.py), parity of the driver paths; where the inter-round gap goes
# (tools/gap_probe.py)
cd /root/repo
timeout -k 10 300 python tools/gap_probe.py --rounds 60 > gpurun_out/gap_r4o.json || exit 1
cat gpurun_out/gap_r4o.json
echo all-done
