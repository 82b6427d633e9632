#!/bin/bash
# Phase 2 of full-size waves software-pipelined by half batches (production, 1) vs not pipelined (variant 48),
# interleaved in one process per config; records must equal production.  (The variants 49 / 50 of the
# committed results were removed after their measurement.)
set -o pipefail
OUT=gpurun_out/${1:-pipe_ab}
mkdir -p $OUT
for c in 2 5 3; do
  timeout -k 10 240 python scripts/variants.py --config $c --variants 1,48 --rounds ${ROUNDS:-20} > $OUT/pipe_c$c.json 2> $OUT/pipe_c$c.err \
    || { echo "config $c failed"; tail -5 $OUT/pipe_c$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/pipe_c$c.json')); print($c, {k: v['ms_median'] for k, v in d.items() if isinstance(v, dict) and 'algo_tbps' in v}, d['calib_stream_read_tbps'])"
done
