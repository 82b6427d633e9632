#!/bin/bash
# Round 4: reference-parity soak on the GPU (more server populations and client scripts than the suite),
# and the driver's torchrun launch at N=2 and N=4 on this one GPU (per-rank device fields).
#   bash scripts/gpu_r4_e.sh <tag>
set -o pipefail
TAG=${1:-r4e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 ./tests/cpp/test_ref_server gpu 10 > $OUT/ref_server_gpu10.log 2>&1 || { tail -20 $OUT/ref_server_gpu10.log; exit 1; }
grep -c "GPU backend) vs reference" $OUT/ref_server_gpu10.log; tail -1 $OUT/ref_server_gpu10.log
timeout -k 10 300 ./tests/cpp/test_ref_client gpu 40 > $OUT/ref_client_gpu40.log 2>&1 || { tail -20 $OUT/ref_client_gpu40.log; exit 1; }
tail -2 $OUT/ref_client_gpu40.log
for N in 2 4; do
  PORT=$((20000 + RANDOM % 20000))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $PORT \
    bench.py --gpus $N --steps 20 --warmup 3 > $OUT/bench_n${N}_torchrun.json 2> $OUT/bench_n${N}_torchrun.err \
    || { echo "n$N failed"; tail -20 $OUT/bench_n${N}_torchrun.err; exit 1; }
  python3 -c "
import json; L=json.load(open('$OUT/bench_n${N}_torchrun.json')); cg=L['correctness_gate']
print($N, L['value'], L['ms_per_step'], cg['every_rank_verified'], cg['every_rank_sha256_gated'], cg['setup_s_max'], cg['peak_rss_mib_max'])"
done
echo r4e-ok
