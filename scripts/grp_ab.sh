#!/bin/bash
# Records of 2 / 4 consecutive 64-slot groups per workgroup written in one burst (variants 23 / 24) vs production,
# on the round-3 final tree; records must equal production.
set -o pipefail
OUT=gpurun_out/${1:-grp_ab}
mkdir -p $OUT
for c in 2 3 5; do
  timeout -k 10 240 python scripts/variants.py --config $c --variants ${VARIANTS:-1,23,24} --rounds ${ROUNDS:-12} > $OUT/grp_c$c.json 2> $OUT/grp_c$c.err \
    || { echo "config $c failed"; tail -5 $OUT/grp_c$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/grp_c$c.json')); print($c, {k: v['ms_median'] for k, v in d.items() if isinstance(v, dict) and 'algo_tbps' in v})"
done
