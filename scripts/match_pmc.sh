#!/bin/bash
# HBM traffic of pn_match_streams' production kernel (match_streams_mask_kernel), the round-3 kernel and
# the production form's loads-only ceiling, under scripts/match_ab.py on C2, counters in their own
# rocprofv3 passes.   bash scripts/match_pmc.sh <tag>
set -o pipefail
TAG=${1:-match_pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="scripts/match_ab.py --configs 2 --rounds 2 --variants 1,13,18"
pass() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o pmc -- python3 $B > $OUT/$name.json 2> $OUT/$name.err \
    || { echo "pass $name failed"; tail -5 $OUT/$name.err; return 1; }
}
pass fetch FETCH_SIZE && pass write WRITE_SIZE && \
pass ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum && \
pass l2 TCC_HIT_sum TCC_MISS_sum || exit 1
python3 scripts/pmc_by_kernel.py $OUT match_streams > $OUT/pmc_by_kernel.json
cat $OUT/pmc_by_kernel.json
