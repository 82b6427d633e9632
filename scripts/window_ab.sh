#!/bin/bash
# Window loads all in flight (production, round 3) vs the serialized form before it (variant 47,
# kSerialWindow), interleaved in one process per config; records of both must equal production.
set -o pipefail
OUT=gpurun_out/${1:-window_ab}
mkdir -p $OUT
for c in 2 3 5; do
  timeout -k 10 240 python scripts/variants.py --config $c --variants 1,47,11 --rounds ${ROUNDS:-15} > $OUT/window_c$c.json 2> $OUT/window_c$c.err \
    || { echo "config $c failed"; tail -5 $OUT/window_c$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/window_c$c.json')); print($c, {k: v['ms_median'] for k, v in d.items() if isinstance(v, dict) and 'algo_tbps' in v})"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/bench.json')); s=d['secondary']
print('c2', d['roofline']['kernel_ms_avg'], d['roofline']['frac'], 'c3', s['c3']['frac'], 'packed', s['c3']['packed_indexed']['frac'], 'c5', s['c5']['frac'],
      'tx', s['tx_fill']['frame_off_2']['frac'], s['tx_fill']['frame_off_14']['frac'], 'verified', d['verified_vs_oracle'])"
