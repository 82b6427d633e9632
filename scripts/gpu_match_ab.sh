#!/bin/bash
# match_streams A/B only:  MATCH_VARIANTS=13,18,34,35 bash scripts/gpu_match_ab.sh <tag>
set -o pipefail
TAG=${1:-match_ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python scripts/match_ab.py --rounds 11 --variants ${MATCH_VARIANTS:-13,18} > $OUT/match_ab.json 2> $OUT/match_ab.err || { echo "match_ab failed"; tail $OUT/match_ab.err; exit 1; }
python3 -c "
import json; M=json.load(open('$OUT/match_ab.json'))
for c in ('c2','c3'):
    print(c, ' '.join(f\"{v}:{r['ms']}\" for v,r in M[c]['variants'].items()))
"
