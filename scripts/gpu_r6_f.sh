#!/bin/bash
# Round 6: the doorbell round trip with a pipelined poll (pn_test_doorbell_echo_pipe: K reads of the bell in flight,
# G x 64 clocks apart) against the one-read poll, three runs.   bash scripts/gpu_r6_f.sh <tag>
set -o pipefail
TAG=${1:-r6f2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in 1 2 3; do
  timeout -k 10 120 ./bench/bench_doorbell 3000 > $OUT/doorbell.$r.json 2> $OUT/doorbell.$r.err || { echo "doorbell rc=$?"; tail $OUT/doorbell.$r.err; exit 1; }
done
python3 - $OUT <<'P'
import json, glob, sys
rows = [json.load(open(f)) for f in sorted(glob.glob(f"{sys.argv[1]}/doorbell.*.json"))]
for k in rows[0]:
    if isinstance(rows[0][k], dict):
        print(f"{k:22s}", " ".join(f"{r[k]['us_median']:6.2f}/{r[k]['us_p90']:6.2f}" for r in rows))
P
