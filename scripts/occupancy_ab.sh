#!/bin/bash
# Production (4 waves/SIMD) vs a 5-wave register budget (variant 52; 96 VGPRs, 16 B/lane of spill), after the
# round-3 window fix and pipelining.  Variant 52 was removed after the measurement (profiles/r03/window/five_waves_c*.json).
set -o pipefail
OUT=gpurun_out/${1:-occ_ab}
mkdir -p $OUT
for c in 3 5 2; do
  timeout -k 10 240 python scripts/variants.py --config $c --variants 1,52 --rounds ${ROUNDS:-15} > $OUT/occ_c$c.json 2> $OUT/occ_c$c.err \
    || { echo "config $c failed"; tail -5 $OUT/occ_c$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/occ_c$c.json')); print($c, {k: v['ms_median'] for k, v in d.items() if isinstance(v, dict) and 'algo_tbps' in v})"
done
