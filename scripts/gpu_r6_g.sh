#!/bin/bash
# Round 6: where a resident-service post spends its time on the device (bench/svc_trace against the -DPN_SVC_TRACE
# build of the library), two runs.   bash scripts/gpu_r6_g.sh <tag>
set -o pipefail
TAG=${1:-r6g2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 120 ./bench/svc_trace 300 > $OUT/trace.$r.json 2> $OUT/trace.$r.err || { echo "svc_trace rc=$?"; tail $OUT/trace.$r.err; exit 1; }
done
python3 - $OUT <<'P'
import json, glob, sys
for f in sorted(glob.glob(f"{sys.argv[1]}/trace.*.json")):
    d = json.load(open(f))
    for k, v in d.items():
        if isinstance(v, dict):
            print(f"{k:24s}", " ".join(f"{kk}={vv}" for kk, vv in v.items()))
P
