#!/bin/bash
# The probe finished after phase 2 (variant 42, kLateProbe) vs production (1), after the window and
# pipelining changes of round 3; no-walk (43) and no-probe (11) ablations beside them.
set -o pipefail
OUT=gpurun_out/${1:-late_ab}
mkdir -p $OUT
for c in 5 3 2; do
  timeout -k 10 240 python scripts/variants.py --config $c --variants 1,42,43,11 --rounds ${ROUNDS:-15} > $OUT/late_c$c.json 2> $OUT/late_c$c.err \
    || { echo "config $c failed"; tail -5 $OUT/late_c$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/late_c$c.json')); print($c, {k: v['ms_median'] for k, v in d.items() if isinstance(v, dict) and 'algo_tbps' in v})"
done
