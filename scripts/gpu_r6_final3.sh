#!/bin/bash
# Round-6 final tree after the service's in-order fix, one pass: host facts, the GPU suite + smoke, the default bench line, a rocprofv3 kernel trace
# of a C2-only run (its rx_classify_kernel average against that line's HIP events), the
# 16-population server soak.  No N=8 launch: the driver runs
# the multi-GPU bench.  Each step has its own time limit; the first failure ends it.
#   bash scripts/gpu_r6_final3.sh <tag>
set -o pipefail
TAG=${1:-r6final3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
{ df -h /dev/shm; free -g; nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; lscpu | grep -E "Model name"; } > $OUT/host.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 \
  || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
timeout -k 10 420 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
python3 -c "import json; L=json.load(open('$OUT/bench.json')); print(json.dumps(L['summary']))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o trace -- \
  python3 bench.py --no-cpu-baseline --no-e2e --no-secondary --steps 50 > $OUT/prof_c2_bench.json 2> $OUT/prof_c2.err || { echo "c2 trace failed"; tail -20 $OUT/prof_c2.err; exit 1; }
find $OUT/prof_c2 -name "*kernel_stats.csv" -exec grep -h "rx_classify_kernel" {} \; | cut -c1-200
python3 -c "import json; L=json.load(open('$OUT/prof_c2_bench.json')); print('c2 traced line', L['roofline']['kernel_ms_avg'], L['roofline']['frac'])"
timeout -k 10 300 ./tests/cpp/test_tcp_server_peer gpu 16 > $OUT/peer16.txt 2>&1 || { echo "peer soak failed"; tail -20 $OUT/peer16.txt; exit 1; }
echo "peer16 identical: $(grep -c 'gpu: handler log identical, TX frames identical' $OUT/peer16.txt)"
echo final-ok
