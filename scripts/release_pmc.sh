#!/bin/bash
# HBM traffic of the release-path classify (header lines only): FETCH_SIZE / WRITE_SIZE / EA request passes, each
# its own rocprofv3 run, then the per-dispatch medians.   bash scripts/release_pmc.sh <tag>
set -o pipefail
TAG=${1:-release_pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o pmc -- python3 scripts/release_pmc_run.py \
    > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $OUT/$name.log; return 1; }
}
pass fetch FETCH_SIZE && pass write WRITE_SIZE && \
pass ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum && \
pass eaw TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, json, os, statistics, sys, collections
out = sys.argv[1]
per = collections.defaultdict(lambda: collections.defaultdict(float))
for sub in ("fetch", "write", "ea", "eaw"):
    for f in glob.glob(os.path.join(out, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = "classify" if "rx_classify" in r["Kernel_Name"] else "calib" if "calib_stream" in r["Kernel_Name"] else None
            if k:
                per[(k, r["Counter_Name"])][r.get("Dispatch_Id")] += float(r["Counter_Value"])
med = {f"{k}:{c}": statistics.median(v.values()) for (k, c), v in per.items()}
n = 1 << 20
factor = n * 2048 / (med["calib:FETCH_SIZE"] * 1024)
read = med["classify:FETCH_SIZE"] * 1024 * factor
write = med["classify:WRITE_SIZE"] * 1024
res = {"frames_per_launch": n, "fetch_correction_factor": round(factor, 4), "hbm_read_bytes_per_launch": int(read),
       "hbm_write_bytes_per_launch": int(write), "read_bytes_per_frame": round(read / n, 2),
       "ea_read_128B_per_frame": round(med.get("classify:TCC_EA0_RDREQ_128B_sum", 0) / n, 4),
       "counters_median_per_dispatch": med}
json.dump(res, open(os.path.join(out, "release_pmc.json"), "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "counters_median_per_dispatch"}))
PY
