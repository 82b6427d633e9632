#!/bin/bash
# Round 5, first GPU session: the GPU suite, then the bench line, then (optional) the TX A/B.  Each step has its
# own time limit; after an abort, a segfault or a time limit nothing more runs (an ordinary test failure, rc 1,
# does not stop the bench).   bash scripts/gpu_r5_a.sh <tag> [tx]
set -o pipefail
TAG=${1:-r5a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
fatal() { case $1 in 0|1) return 1 ;; *) return 0 ;; esac; }
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?
  echo "$name rc=$rc"
  if fatal $rc; then echo "stopping after $name (rc $rc)"; exit $rc; fi
  return 0
}
step tests 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step bench 420 python bench.py
if [ "$2" = tx ]; then
  for off in 14 2; do
    step tx_ab_off$off 300 python scripts/tx_variants.py --frame-off $off --variants 40,50,51,52,41 --rotate 4 --rounds 9
  done
fi
tail -3 $OUT/tests.out
