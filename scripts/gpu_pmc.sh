#!/bin/bash
# HBM traffic of the production kernel under the bench's own conditions (rotating
# resident batches), counters in their own rocprofv3 passes (kernel-trace/stats
# never combined with --pmc).  bench.py's ceilings() runs the calibration stream
# read of a known byte count in the same process (FETCH_SIZE correction).
set -o pipefail
TAG=${1:-pmc}
CFG=${2:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-secondary --stream-ceiling-only"
pass() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o pmc -- python3 $B > $OUT/$name.json 2> $OUT/$name.err \
    || { echo "pass $name failed"; tail -5 $OUT/$name.err; return 1; }
}
pass fetch FETCH_SIZE && pass write WRITE_SIZE && \
pass ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum && \
pass eaw TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_DRAM_sum && \
pass l2 TCC_HIT_sum TCC_MISS_sum || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $B > $OUT/trace.json 2> $OUT/trace.err || echo "trace pass failed (non-fatal)"
find $OUT/trace -name "*kernel_stats.csv" -exec cat {} \;
cat $OUT/fetch.json
