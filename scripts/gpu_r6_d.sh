#!/bin/bash
# Round 6: large service posts on independent helper grids -- the service tests, then the sizing sweep.
#   bash scripts/gpu_r6_d.sh <tag>
set -o pipefail
TAG=${1:-r6d}
OUT=gpurun_out/$TAG
mkdir -p $OUT
fatal() { case $1 in 0|1) return 1 ;; *) return 0 ;; esac; }
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?
  echo "$name rc=$rc"
  if fatal $rc; then echo "stopping after $name (rc $rc)"; tail -30 $OUT/$name.out; exit $rc; fi
  return 0
}
step service 400 python -u -m pytest tests/test_gpu_service.py tests/test_gpu_links.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -3 $OUT/service.out
step sizing 300 python scripts/service_sizing.py --waves 64,576,1088,2112,3136
cat $OUT/sizing.out
