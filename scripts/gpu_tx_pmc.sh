#!/bin/bash
# HBM traffic of the TX fill kernels, one rocprofv3 --pmc pass per counter group
# (never combined with tracing).  bash scripts/gpu_tx_pmc.sh <tag> <frame_off> [--phase2]
set -o pipefail
TAG=${1:-txpmc}; OFF=${2:-2}; EXTRA=$3
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P="scripts/tx_pmc_probe.py --frame-off $OFF $EXTRA"
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o pmc -- python3 $P > $OUT/$name.log 2>&1 \
    || { echo "pass $name failed"; tail -5 $OUT/$name.log; return 1; }
}
pass fetch FETCH_SIZE && pass write WRITE_SIZE && \
pass ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum && \
pass eaw TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, os, statistics, sys, json
root = sys.argv[1]
res = {}
for d in ("fetch", "write", "ea", "eaw"):
    per = {}
    for f in glob.glob(os.path.join(root, d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].split("::")[-1].split("<")[0] + ("<" + r["Kernel_Name"].split("<", 1)[1].split(">")[0] + ">" if "<" in r["Kernel_Name"] else "")
            did = r.get("Dispatch_Id") or r.get("Correlation_Id")
            per.setdefault((k, r["Counter_Name"]), {}).setdefault(did, 0.0)
            per[(k, r["Counter_Name"])][did] += float(r["Counter_Value"])
    for (k, c), v in per.items():
        res.setdefault(k, {})[c] = statistics.median(v.values())
print(json.dumps(res, indent=1))
PY
