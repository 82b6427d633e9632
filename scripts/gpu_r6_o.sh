#!/bin/bash
# Round 6: the device-mailbox service's steps on the device (make svc_trace: the measurement build), two runs.
#   bash scripts/gpu_r6_o.sh <tag>
set -o pipefail
TAG=${1:-r6o}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 120 ./bench/svc_trace 300 > $OUT/trace.$r.json 2> $OUT/trace.$r.err || { echo "rc=$?"; cat $OUT/trace.$r.err; exit 1; }
  cat $OUT/trace.$r.json
done
