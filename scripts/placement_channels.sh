#!/bin/bash
# Per-TCC-channel (x XCD) counters of the C2 kernel per HBM placement: rocprofv3 --pmc with JSON output (one
# record per counter instance), 12 buffers per process (scripts/placement_pmc.py run), then `channels`.
#   bash scripts/placement_channels.sh <tag>
set -o pipefail
TAG=${1:-placement_channels}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for counters in "TCC_EA0_RDREQ TCC_EA0_RDREQ_LEVEL" "TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $counters --output-format json -d $OUT/p$i -o pmc -- \
    python3 scripts/placement_pmc.py run $OUT/p$i.run.json 12 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 scripts/placement_pmc.py channels $OUT > $OUT/channels.json && echo channels-ok
