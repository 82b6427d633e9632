#!/bin/bash
# PMC passes for HBM traffic (counters in their own runs, kernel-trace/stats only).
set -o pipefail
TAG=${1:-pmc}
CFG=${2:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o pmc -- python3 scripts/pmc_probe.py --config $CFG > $OUT/probe_fetch.txt 2> $OUT/fetch.err || { echo "fetch pass failed"; tail -20 $OUT/fetch.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o pmc -- python3 scripts/pmc_probe.py --config $CFG > $OUT/probe_write.txt 2> $OUT/write.err || { echo "write pass failed"; tail -20 $OUT/write.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $OUT/ea -o pmc -- python3 scripts/pmc_probe.py --config $CFG > /dev/null 2> $OUT/ea.err || echo "ea pass failed (non-fatal)"
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/eaw -o pmc -- python3 scripts/pmc_probe.py --config $CFG > /dev/null 2> $OUT/eaw.err || echo "eaw pass failed (non-fatal)"
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/l2 -o pmc -- python3 scripts/pmc_probe.py --config $CFG > $OUT/probe_l2.txt 2> $OUT/l2.err || echo "l2 pass failed (non-fatal)"
cat $OUT/probe_fetch.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 scripts/pmc_probe.py --config $CFG --reps 10 > /dev/null 2> $OUT/trace.err || echo "trace pass failed (non-fatal)"
find $OUT/trace -name "*kernel_stats.csv" -exec cat {} \;
