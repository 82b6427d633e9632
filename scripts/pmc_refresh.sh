#!/bin/bash
# Refresh profiles/pmc_traffic.json: the bench's workloads (scripts/pmc_workloads.py) under rocprofv3, one
# --pmc pass per counter group (never combined with tracing), then a kernel-trace pass of the same program.
# Each pass is its own process with its own time limit; the first failure ends the script.
#   bash scripts/pmc_refresh.sh <tag> [--uncached]
# then, in the container:  python3 scripts/pmc_refresh.py gpurun_out/<tag>
set -o pipefail
TAG=${1:-pmc_refresh}
EXTRA=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
pass() {  # name, counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o pmc -- \
    python3 scripts/pmc_workloads.py --out $OUT/$name $EXTRA > $OUT/$name.log 2>&1 \
    || { echo "pass $name failed"; tail -5 $OUT/$name.log; return 1; }
  echo "pass $name ok"
}
pass fetch FETCH_SIZE && pass write WRITE_SIZE && \
pass ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum && \
pass eaw TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_DRAM_sum || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- \
  python3 scripts/pmc_workloads.py --out $OUT/trace $EXTRA > $OUT/trace.log 2>&1 || { echo "trace pass failed"; exit 1; }
echo "trace ok"
