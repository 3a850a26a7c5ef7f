cd /root/repo
for f in 256 128 8 16 32; do
  timeout -k 10 60 python -u tools/probe.py --phase solve --reps 3 --blocks 1 --flags $f > gpurun_out/l.json || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/l.json')); print($f, round(d['solve']['ms'],4), d['steps_max'], round(d['solve']['ms']*1e-3*2.4e9/d['steps_max'],1))"
done
