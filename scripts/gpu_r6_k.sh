#!/bin/bash
# Round 6: where the drop-in server's host time goes now (the sampler over the pipelined resident GPU leg, the
# reference's server and the twin's dispatch, on the current engine), and three resident_pair rounds beside it.
#   bash scripts/gpu_r6_k.sh <tag>
set -o pipefail
TAG=${1:-r6k}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0|1) return 1 ;; *) return 0 ;; esac; }
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?
  echo "$name rc=$rc"
  if fatal $rc; then echo "stopping after $name (rc $rc)"; tail -30 $OUT/$name.out; exit $rc; fi
  return 0
}
PN_SAMPLE=$OUT/samp step sample_pair 120 ./bench/bench_tcp_server 256 4000 resident_pair
PN_SAMPLE=$OUT/samp step sample_twin 120 ./bench/bench_tcp_server 256 4000 twin_timed
for t in gpu reference twin; do
  python3 scripts/sample_report.py bench/bench_tcp_server $OUT/samp.$t --top 60 --lines > $OUT/profile_$t.txt 2>&1
done
for r in 1 2 3; do step pair.$r 120 ./bench/bench_tcp_server 256 3000 resident_pair; done
tail -c 600 $OUT/pair.1.out
