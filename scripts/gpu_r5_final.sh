#!/bin/bash
# Round-5 final tree, one pass: host facts, the GPU suite + smoke, the default bench line, a rocprofv3 kernel trace of
# the full bench (its kernel averages against the line's HIP events), and the driver's N=8 torchrun launch with the
# end-to-end host-ring leg rehearsed on this one GPU.  Each step has its own time limit; the first failure ends it.
#   bash scripts/gpu_r5_final.sh <tag>
set -o pipefail
TAG=${1:-r5final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
{ df -h /dev/shm; free -g; nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; } > $OUT/host.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 \
  || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
python3 -c "import json; L=json.load(open('$OUT/bench.json')); print(json.dumps(L['summary']))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_full -o trace -- \
  python3 bench.py --no-cpu-baseline --steps 50 > $OUT/prof_full_bench.json 2> $OUT/prof_full.err || { echo "full trace failed"; tail -20 $OUT/prof_full.err; exit 1; }
find $OUT/prof_full -name "*kernel_stats.csv" -exec grep -h "rx_classify_kernel\|match_streams_mask\|tx_fill_kernel" {} \; | cut -c1-160
python3 -c "import json; L=json.load(open('$OUT/prof_full_bench.json')); print('traced line', L['roofline']['kernel_ms_avg'], L['roofline']['frac'])"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 8 --steps 10 --warmup 2 --batches 2 --e2e > $OUT/n8_e2e.json 2> $OUT/n8_e2e.err || { echo "n8 e2e failed"; tail -20 $OUT/n8_e2e.err; exit 1; }
python3 -c "
import json; L=[json.loads(l) for l in open('$OUT/n8_e2e.json') if l.startswith('{')][-1]
print('n8', L['value'], L['verified_vs_oracle'], json.dumps(L.get('e2e_host_ring', {}))[:600])"
echo final-ok
