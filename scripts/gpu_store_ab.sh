#!/bin/bash
# RX record-store cost split: production (1), no store (18), every store into 16 KiB (49), store policies (5 default,
# 7 nt, 8 plain global), on C2 and C3.   bash scripts/gpu_store_ab.sh <tag>
set -o pipefail
TAG=${1:-store_ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for c in ${RX_CONFIGS:-2 3}; do
  timeout -k 10 300 python scripts/variants.py --config $c --rounds 11 --variants ${RX_VARIANTS:-1,18,49,5,7,8} > $OUT/c$c.json 2> $OUT/c$c.err \
    || { echo "variants c$c failed"; tail $OUT/c$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/c$c.json'))
print('c$c', ' '.join(f\"{k}:{v['ms_median']}\" for k,v in d.items() if isinstance(v, dict)))
"
done
