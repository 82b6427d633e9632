#!/bin/bash
# Run-length hint probe (variant 46) A/B against production (1), home-slot-only (43) and no probe (11),
# interleaved in one process per config (scripts/variants.py; records of 1 and 46 must equal production).
set -o pipefail
OUT=gpurun_out/${1:-hint_ab}
mkdir -p $OUT
for c in 5 3 2; do
  timeout -k 10 240 python scripts/variants.py --config $c --variants 1,46,43,11 --rounds ${ROUNDS:-15} > $OUT/hint_c$c.json 2> $OUT/hint_c$c.err \
    || { echo "config $c failed"; tail -5 $OUT/hint_c$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/hint_c$c.json')); print($c, {k: v['ms_median'] for k, v in d.items() if isinstance(v, dict) and 'algo_tbps' in v})"
done
