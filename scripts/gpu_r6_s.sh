#!/bin/bash
# Round 6: the drop-in server's GPU tests, the host-mailbox fallback among them.   bash scripts/gpu_r6_s.sh <tag>
set -o pipefail
TAG=${1:-r6s}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_tcp_server.py -m gpu -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
grep -E "PASSED|FAILED" $OUT/tests.log; tail -1 $OUT/tests.log
