#!/bin/bash
# HBM traffic of pn_match_streams (both kernel forms) and its same-pattern ceiling (the first 64 /
# 128 B of every slot, calib_slot_read) under scripts/bench_streams.py on C2, counters in their own
# rocprofv3 passes; plus a kernel-trace pass.  bash scripts/streams_pmc.sh <tag>
set -o pipefail
TAG=${1:-streams_pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="scripts/bench_streams.py --configs 2 --rounds 3 --policies"
pass() {  # name, counters...
  local name=$1; shift
  timeout -k 10 180 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o pmc -- python3 $B > $OUT/$name.json 2> $OUT/$name.err \
    || { echo "pass $name failed"; tail -5 $OUT/$name.err; return 1; }
}
pass fetch FETCH_SIZE && pass write WRITE_SIZE && \
pass ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum && \
pass l2 TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $B > $OUT/trace.json 2> $OUT/trace.err || { echo "trace pass failed"; exit 1; }
python3 scripts/pmc_by_kernel.py $OUT match_streams calib > $OUT/pmc_by_kernel.json
cat $OUT/pmc_by_kernel.json
