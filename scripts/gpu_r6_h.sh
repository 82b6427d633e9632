#!/bin/bash
# Round 6: a service A/B -- the service and link tests, the post round trips (bench_signal) of the previous library
# (ab_libs/old) and this one, interleaved, and the device step clocks (svc_trace).  Used for the tagged-line publish
# (r6h2) and the XCD-aware wave ranks (r6h3).   bash scripts/gpu_r6_h.sh <tag>
set -o pipefail
TAG=${1:-r6h2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
fatal() { case $1 in 0|1) return 1 ;; *) return 0 ;; esac; }
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?
  echo "$name rc=$rc"
  if fatal $rc; then echo "stopping after $name (rc $rc)"; tail -30 $OUT/$name.out; exit $rc; fi
  return 0
}
step service 400 python -u -m pytest tests/test_gpu_service.py tests/test_gpu_links.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -3 $OUT/service.out
grep -q " passed" $OUT/service.out && ! grep -q "failed" $OUT/service.out || { echo "service tests not green"; exit 1; }
for r in 1 2 3; do
  LD_LIBRARY_PATH=$PWD/ab_libs/old step signal_old.$r 120 ./bench/bench_signal 300
  step signal_new.$r 120 ./bench/bench_signal 300
done
step trace 120 ./bench/svc_trace 300
python3 - $OUT <<'P'
import json, glob, sys
out = sys.argv[1]
for tag in ("old", "new"):
    rows = [json.load(open(f)) for f in sorted(glob.glob(f"{out}/signal_{tag}.*.out"))]
    for leg in ("resident", "zero_copy", "resident_release_path", "zero_copy_release_path"):
        print(tag, f"{leg:24s}", " ".join(f"{n}:" + "/".join(f"{r[leg][n]['service_us']:.2f}" for r in rows) for n in ("64", "512", "1024")),
              "eq", all(r[leg][n]["records_equal"] for r in rows for n in ("64", "512", "1024")))
d = json.load(open(f"{out}/trace.out"))
for k, v in d.items():
    if isinstance(v, dict): print(f"{k:24s}", " ".join(f"{kk}={vv}" for kk, vv in v.items()))
P
