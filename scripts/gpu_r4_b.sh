#!/bin/bash
# Round 4: match_streams forms, parity (numpy) then interleaved A/B.   bash scripts/gpu_r4_b.sh <tag>
set -o pipefail
TAG=${1:-r4b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_match_streams.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/match_tests.log 2>&1 \
  || { tail -30 $OUT/match_tests.log; exit 1; }
tail -1 $OUT/match_tests.log
timeout -k 10 400 python scripts/match_ab.py $MATCH_AB_ARGS > $OUT/match_ab.json 2> $OUT/match_ab.err || { echo "match_ab failed"; tail $OUT/match_ab.err; exit 1; }
python3 -c "
import json; M=json.load(open('$OUT/match_ab.json'))
for c in ('c2','c3'):
    print(c, ' '.join(f\"{v}:{r['ms']}\" for v,r in M[c]['variants'].items()))
"
echo r4b-ok
