#!/bin/bash
# Round 4: match_streams micro-variants A/B, and the C2-only kernel trace + bench line for the roofline
# evidence.   bash scripts/gpu_r4_d.sh <tag>
set -o pipefail
TAG=${1:-r4d}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_match_streams.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/match_tests.log 2>&1 \
  || { tail -30 $OUT/match_tests.log; exit 1; }
tail -1 $OUT/match_tests.log
timeout -k 10 400 python scripts/match_ab.py --rounds 11 --variants 13,18,33 > $OUT/match_ab.json 2> $OUT/match_ab.err || { echo "match_ab failed"; tail $OUT/match_ab.err; exit 1; }
python3 -c "
import json; M=json.load(open('$OUT/match_ab.json'))
for c in ('c2','c3'):
    print(c, ' '.join(f\"{v}:{r['ms']}\" for v,r in M[c]['variants'].items()))
"
echo skip-trace && exit 0
  python3 bench.py --no-cpu-baseline --no-e2e --no-secondary --steps 50 > $OUT/prof_c2_bench.json 2> $OUT/prof_c2.err || { echo "c2 trace failed"; tail -20 $OUT/prof_c2.err; exit 1; }
find $OUT/prof_c2 -name "*kernel_stats.csv" -exec grep -h "rx_classify_kernel" {} \; | cut -c1-200
python3 -c "import json; L=json.load(open('$OUT/prof_c2_bench.json')); print('line', L['roofline']['kernel_ms_avg'], L['roofline']['frac'])"
echo r4d-ok
