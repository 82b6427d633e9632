#!/bin/bash
# EA read requests per variant (one --pmc pass each; counters only, no tracing).
set -o pipefail
TAG=${1:-vtraffic}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for V in "$@"; do
  timeout -k 10 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum --output-format csv -d $OUT/v$V -o pmc -- python3 scripts/pmc_probe.py --variant $V > /dev/null 2> $OUT/v$V.err || { echo "variant $V pass failed"; tail -5 $OUT/v$V.err; exit 1; }
done
python3 - "$OUT" "$@" <<'PY'
import csv, glob, statistics, sys
out = sys.argv[1]
for v in sys.argv[2:]:
    agg = {}
    for f in glob.glob(f"{out}/v{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "rx_classify" not in r["Kernel_Name"]:
                continue
            agg.setdefault(r["Counter_Name"], {}).setdefault(r.get("Dispatch_Id"), 0.0)
            agg[r["Counter_Name"]][r.get("Dispatch_Id")] += float(r["Counter_Value"])
    print("variant", v, {k: statistics.median(d.values()) / 1048576 for k, d in agg.items()}, "(per frame)")
PY
