#!/bin/bash
# Round 6: the service's posts taken strictly in order from their own slot -- the ring-reuse soak in both mailbox
# modes, the service / link / server GPU tests (the host-mailbox server test among them), then the peer test with
# PN_SERVICE_HOST_MAILBOX three more times.   bash scripts/gpu_r6_t.sh <tag>
set -o pipefail
TAG=${1:-r6t}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_service.py tests/test_gpu_links.py tests/test_tcp_server.py -m gpu -v \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|Error|passed|failed" $OUT/tests.log | tail -8
[ $rc -le 1 ] || exit $rc
for r in 1 2 3; do
  PN_SERVICE_HOST_MAILBOX=1 timeout -k 10 200 ./tests/cpp/test_tcp_server_peer gpu 2 > $OUT/peer_host.$r.txt 2>&1; rc=$?
  echo "peer host mailbox run $r rc=$rc identical=$(grep -c 'gpu: handler log identical, TX frames identical' $OUT/peer_host.$r.txt)"
  [ $rc -le 1 ] || exit $rc
done
