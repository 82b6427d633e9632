#!/bin/bash
# pn_tx_fill's two phases (tuning variant 40) vs one in-place launch (41) at the product's launch shape, over 4
# rotating batches (the bench's steady state), at frame_off 14 (efvitcp's SendBuf layout) and 2, two runs each.
#   bash scripts/gpu_tx_inplace_ab.sh <tag>
set -o pipefail
TAG=${1:-tx_inplace}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for off in 14 2; do
    timeout -k 10 300 python scripts/tx_variants.py --frame-off $off --variants 40,41 --rotate 4 --rounds 12 \
      > $OUT/off${off}_run$r.json 2> $OUT/err.log || { echo "variants failed"; tail $OUT/err.log; exit 1; }
  done
done
python3 -c "
import json
for r in (1, 2):
    for off in (14, 2):
        d=json.load(open('$OUT/off%d_run%d.json' % (off, r))); print(off, r, {k:v['ms_median'] for k,v in d.items() if isinstance(v,dict) and 'product' in k})"
