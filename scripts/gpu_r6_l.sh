#!/bin/bash
# Round 6: can the host post into device memory?  The doorbell round trip with the bell in VRAM written through the
# large BAR (uncached and fine-grained allocations) beside the host-memory bell, three runs.   bash scripts/gpu_r6_l.sh <tag>
set -o pipefail
TAG=${1:-r6l}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in 1 2 3; do
  timeout -k 10 60 ./bench/bench_doorbell 2000 device > $OUT/doorbell_dev.$r.json 2> $OUT/doorbell_dev.$r.err || { echo "rc=$? run $r"; cat $OUT/doorbell_dev.$r.json $OUT/doorbell_dev.$r.err; exit 1; }
  cat $OUT/doorbell_dev.$r.json
done
