#!/bin/bash
# Round 6: the drop-in server soak on the device-mailbox service -- 16 peer populations x 8 RX modes (the resident
# modes among them), GPU backend against the twin.   bash scripts/gpu_r6_q.sh <tag>
set -o pipefail
TAG=${1:-r6q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 ./tests/cpp/test_tcp_server_peer gpu 16 > $OUT/peer16.txt 2>&1 || { echo "rc=$?"; tail -30 $OUT/peer16.txt; exit 1; }
grep -c "gpu: handler log identical, TX frames identical" $OUT/peer16.txt
tail -1 $OUT/peer16.txt
