#!/bin/bash
# The driver's N=8 launch on one MI355X with the final tree (8 ranks time-sharing the device): every rank's C4
# shard gated, per-rank device/setup/RSS fields.   bash scripts/gpu_r4_n8_final.sh <tag>
set -o pipefail
TAG=${1:-r4n8final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PORT=$((20000 + RANDOM % 20000))
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $PORT \
  bench.py --gpus 8 --steps 20 --warmup 3 > $OUT/bench_n8_torchrun.json 2> $OUT/bench_n8_torchrun.err \
  || { echo "n8 failed"; tail -30 $OUT/bench_n8_torchrun.err; exit 1; }
python3 -c "
import json; L=json.load(open('$OUT/bench_n8_torchrun.json')); cg=L['correctness_gate']
print(L['value'], L['ms_per_step'], L['verified_vs_oracle'], cg['every_rank_verified'], cg['every_rank_sha256_gated'], cg['setup_s_max'], cg['peak_rss_mib_max'])"
echo n8-ok
