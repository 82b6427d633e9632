#!/bin/bash
# Round 6: the post counter's wrap -- the service tests (the wrap test included) and the drop-in server's GPU tests
# (every RX mode, and the resident modes with the counter started below 2^32).   bash scripts/gpu_r6_i.sh <tag>
set -o pipefail
TAG=${1:-r6i}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_service.py tests/test_tcp_server.py tests/test_gpu_links.py -m gpu -v \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
