#!/bin/bash
# Round-4 final tree: GPU suite + smoke, the default bench line, a rocprofv3 kernel trace of the full bench
# (its rx_classify_kernel and match_streams_mask_kernel averages against the line's HIP events), and the
# match_streams PMC passes.   bash scripts/gpu_r4_final.sh <tag>
set -o pipefail
TAG=${1:-r4final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 \
  || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
python3 -c "
import json; L=json.load(open('$OUT/bench.json')); s=L['secondary']
print('C2', L['roofline']['kernel_ms_avg'], L['roofline']['frac'], 'c4_shard', s['c4_shard']['kernel_ms'], s['c4_shard']['frac'])
m=s['match_streams']; print('match', m['kernel_ms'], m['frac'], m['kernel_vs_gather_ceiling'], m['kernel_vs_loads_and_stores_ceiling'], m['first_65536_ids_vs_numpy'])
print('c3', s['c3']['frac'], 'c5', s['c5']['frac'], 'tx', s['tx_fill']['frame_off_2']['frac'], s['tx_fill']['frame_off_14']['frac'])
"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_full -o trace -- \
  python3 bench.py --no-cpu-baseline --no-e2e --steps 50 > $OUT/prof_full_bench.json 2> $OUT/prof_full.err || { echo "full trace failed"; tail -20 $OUT/prof_full.err; exit 1; }
find $OUT/prof_full -name "*kernel_stats.csv" -exec grep -h "rx_classify_kernel\|match_streams_mask\|tx_fill_kernel" {} \; | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o trace -- \
  python3 bench.py --no-cpu-baseline --no-e2e --no-secondary --steps 50 > $OUT/prof_c2_bench.json 2> $OUT/prof_c2.err || { echo "c2 trace failed"; tail -20 $OUT/prof_c2.err; exit 1; }
find $OUT/prof_c2 -name "*kernel_stats.csv" -exec grep -h "rx_classify_kernel" {} \; | cut -c1-200
python3 -c "import json; L=json.load(open('$OUT/prof_c2_bench.json')); print('c2 traced line', L['roofline']['kernel_ms_avg'], L['roofline']['frac'])"
echo final-ok
