#!/bin/bash
# Round 6: the whole GPU suite and the smoke on the tree after the depth-2 pipeline and the post-id wrap fix.
#   bash scripts/gpu_r6_j.sh <tag>
set -o pipefail
TAG=${1:-r6j}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 \
  || { tail -60 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
