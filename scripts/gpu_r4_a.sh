#!/bin/bash
# Round 4, first GPU pass: the whole GPU suite (with the new reference-server parity and notify-counter
# tests), the default bench line (now with secondary.c4_shard), and the driver's N=8 launch rehearsed on
# this one GPU at full C4 size (8 ranks x 4 x 4-GiB shards).
#   bash scripts/gpu_r4_a.sh <tag>
set -o pipefail
TAG=${1:-r4a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 \
  || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
head -c 600 $OUT/bench.json; echo
timeout -k 10 300 python scripts/match_ab.py > $OUT/match_ab.json 2> $OUT/match_ab.err || { echo "match_ab failed"; tail $OUT/match_ab.err; exit 1; }
PORT=$((20000 + RANDOM % 20000))
( while sleep 30; do free -g | awk 'NR==2{print "host mem used GiB", $3}'; done ) > $OUT/n8_mem.log 2>&1 &
MON=$!
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $PORT \
  bench.py --gpus 8 --steps 20 --warmup 3 > $OUT/bench_n8_torchrun.json 2> $OUT/bench_n8_torchrun.err
RC=$?
kill $MON
[ $RC -eq 0 ] || { echo "n8 failed rc=$RC"; tail -30 $OUT/bench_n8_torchrun.err; exit 1; }
head -c 1500 $OUT/bench_n8_torchrun.json; echo
echo r4a-ok
