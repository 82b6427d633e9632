#!/bin/bash
# EA read-request size counters (exact bytes = 32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B?), own passes.
set -o pipefail
TAG=${1:-traffic}
CFG=${2:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $OUT/rdreq -o pmc -- python3 scripts/pmc_probe.py --config $CFG > $OUT/probe.txt 2> $OUT/rdreq.err || { echo "rdreq pass failed"; tail -20 $OUT/rdreq.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/dram -o pmc -- python3 scripts/pmc_probe.py --config $CFG > /dev/null 2> $OUT/dram.err || { echo "dram pass failed"; tail -20 $OUT/dram.err; }
python3 - <<PY
import csv, glob, statistics
for d in ("rdreq", "dram"):
    rows = []
    for f in glob.glob("$OUT/%s/**/*counter_collection.csv" % d, recursive=True):
        rows += list(csv.DictReader(open(f)))
    agg = {}
    for r in rows:
        k = (r["Kernel_Name"][:32], r["Counter_Name"])
        agg.setdefault(k, {}).setdefault(r.get("Dispatch_Id"), 0.0)
        agg[k][r.get("Dispatch_Id")] += float(r["Counter_Value"])
    for k, v in sorted(agg.items()):
        print(k, statistics.median(v.values()))
PY
