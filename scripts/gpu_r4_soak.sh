#!/bin/bash
# Reference-parity soak on the GPU with the final handlers (sendv / writeSome / sendable figures logged):
# 10 + 10 server populations, 40 client scripts, and the stream test in both delivery modes.
#   bash scripts/gpu_r4_soak.sh <tag>
set -o pipefail
TAG=${1:-r4soak}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 ./tests/cpp/test_ref_server gpu 10 > $OUT/ref_server_gpu10.log 2>&1 || { tail -20 $OUT/ref_server_gpu10.log; exit 1; }
grep -c "GPU backend) vs reference" $OUT/ref_server_gpu10.log; tail -1 $OUT/ref_server_gpu10.log
timeout -k 10 300 ./tests/cpp/test_ref_client gpu 40 > $OUT/ref_client_gpu40.log 2>&1 || { tail -20 $OUT/ref_client_gpu40.log; exit 1; }
tail -2 $OUT/ref_client_gpu40.log
timeout -k 10 120 ./tests/cpp/test_gpu_tcp_stream oracle/_ref/libref_tcpstream.so > $OUT/gpu_tcp_stream.log 2>&1 || { tail -20 $OUT/gpu_tcp_stream.log; exit 1; }
tail -1 $OUT/gpu_tcp_stream.log
echo soak-ok
