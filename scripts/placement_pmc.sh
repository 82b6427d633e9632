#!/bin/bash
# Counters of the C2 kernel per HBM placement (scripts/placement_pmc.py), one rocprofv3 --pmc pass
# per counter set (each a separate process: its own placements, each classified as it comes).
#   bash scripts/placement_pmc.sh <tag> "<counters pass 1>" "<counters pass 2>" ...
set -o pipefail
TAG=${1:-placement}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for counters in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $counters --output-format csv -d $OUT/p$i -o pmc -- \
    python3 scripts/placement_pmc.py run $OUT/p$i.run.json 8 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 scripts/placement_pmc.py summarize $OUT > $OUT/summary.json && cat $OUT/summary.json
