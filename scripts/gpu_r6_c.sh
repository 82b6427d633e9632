#!/bin/bash
# Round 6: the chain pass's cost -- post round trips with and without links (bench_signal), and the drop-in server
# with and without them beside the reference (host A/B).   bash scripts/gpu_r6_c.sh <tag>
set -o pipefail
TAG=${1:-r6c}
OUT=gpurun_out/$TAG
mkdir -p $OUT
fatal() { case $1 in 0|1) return 1 ;; *) return 0 ;; esac; }
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?
  echo "$name rc=$rc"
  if fatal $rc; then echo "stopping after $name (rc $rc)"; tail -30 $OUT/$name.err; exit $rc; fi
  return 0
}
step signal 120 ./bench/bench_signal 300
python3 -c "
import json; d=json.load(open('$OUT/signal.out'))
for k in ('zero_copy','zero_copy_release_path'):
    print(k, {n: (v['service_us'], v['service_linked_us']) for n, v in d[k].items()})"
step links_gpu 200 python -u -m pytest tests/test_gpu_links.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -2 $OUT/links_gpu.out
step host_ab 400 bash scripts/host_ab.sh $TAG/ab 4 scratch_ab/srv_B scratch_ab/srv_C
cat $OUT/host_ab.out
python3 - $OUT/ab <<'P'
import json, glob, sys, statistics
d=[json.load(open(x)) for x in sorted(glob.glob(f"{sys.argv[1]}/srv_C.pair.*.json"))]
for k in ("gpu_rxbatch_512_pipelined_resident_release_path","gpu_rxbatch_512_pipelined_resident_unlinked_release_path","reference_server_release_build"):
    print(k, statistics.median(x[k]["mframes_per_s"] for x in d))
P
