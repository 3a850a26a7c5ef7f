#!/bin/bash
# GPU-box session helper: run the steps named on the command line in order,
# each under its own time limit, logs under gpurun_out/.  A step that faults,
# aborts or times out (exit status other than 0 or 1) ends the session.
#   tools/gpu_run.sh tests probe bench
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "== stopping after $name (rc=$rc)"
    exit $rc
  fi
  return 0
}
for s in "$@"; do
  case $s in
    tests) step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    probe) step probe_sp 180 python -u tools/probe.py --reps 3 &&
           step probe_vt 180 python -u tools/probe.py --reps 3 --flags 32 ;;
    bench) step bench 600 python -u bench.py ;;
    bench_twins) step bench_twins 600 python -u bench.py --mode twins ;;
    bench_triplets) step bench_triplets 600 python -u bench.py --mode triplets ;;
    bench_n2000) step bench_n2000 600 python -u bench.py --n 2000 --steps 5 --warmup 1 --no-cpu-baseline ;;
    bench_n2000cpu) step bench_n2000cpu 900 python -u bench.py --n 2000 --steps 5 --warmup 1 --b1-seconds 20 ;;
    bench_twins3000) step bench_twins3000 900 python -u bench.py --mode twins --n 3000 --steps 5 --warmup 1 --b1-seconds 30 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
