# dev: tools/diag_round.py under several libraries (abl/<name>.so), stop at the first failure
#   tools/diag_libs.sh "diag args" lib1 lib2 ...
set -o pipefail
ARGS=$1; shift
for L in "$@"; do
  SANTA_HIP_LIB=abl/$L.so timeout -k 10 120 python tools/diag_round.py $ARGS >> gpurun_out/r06_diag.jsonl 2>> gpurun_out/r06_diag.err || exit 1
  tail -1 gpurun_out/r06_diag.jsonl | cut -c1-300
done
