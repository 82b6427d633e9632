#!/bin/bash
# TX fill: the product's two phases (40) vs the same with the window loads serialized as before round 3
# (43), frame_off 2 and 14, 4 rotating batches, interleaved in one process, both orders; frames must equal
# production.
set -o pipefail
OUT=gpurun_out/${1:-tx_window_ab}
mkdir -p $OUT
for off in 2 14; do
  for order in ${ORDERS:-40,43 43,40}; do
    timeout -k 10 240 python scripts/tx_variants.py --frame-off $off --variants $order --rotate 4 --rounds 12 --reps 20 \
      > $OUT/tx_window_off${off}_${order/,/_}.json 2> $OUT/tx_window_off${off}.err || { echo "off $off failed"; tail -5 $OUT/tx_window_off$off.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/tx_window_off${off}_${order/,/_}.json')); print($off, '$order', {k: v.get('ms_median') for k, v in d.items() if isinstance(v, dict)})"
  done
done
