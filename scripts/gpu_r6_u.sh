#!/bin/bash
# Round 6: the default bench line with the server placements in three interleaved rounds (median legs).
#   bash scripts/gpu_r6_u.sh <tag>
set -o pipefail
TAG=${1:-r6u}
OUT=gpurun_out/$TAG
mkdir -p $OUT
start=$(date +%s)
timeout -k 10 420 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
echo "bench seconds: $(( $(date +%s) - start ))"
python3 -c "import json; L=json.load(open('$OUT/bench.json')); print(json.dumps(L['summary']))"
