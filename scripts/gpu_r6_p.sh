#!/bin/bash
# Round 6, measurement only: what the service's per-post system acquire costs -- bench_signal with the product
# library vs a build without that fence (ab_libs/noacq, never shipped: without it a post could read stale lines),
# four interleaved rounds.   bash scripts/gpu_r6_p.sh <tag>
set -o pipefail
TAG=${1:-r6p}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in 1 2 3 4; do
  timeout -k 10 120 ./bench/bench_signal 600 > $OUT/sig_prod.$r.out 2>&1 || exit 1
  LD_LIBRARY_PATH=$PWD/ab_libs/noacq timeout -k 10 120 ./bench/bench_signal 600 > $OUT/sig_noacq.$r.out 2>&1 || exit 1
done
python3 - $OUT <<'P'
import json, glob, sys, statistics
o = sys.argv[1]
def load(pat): return [json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob(f"{o}/{pat}"))]
rows = {t: load(f"sig_{t}.*.out") for t in ("prod", "noacq")}
for leg in ("resident", "zero_copy", "resident_release_path", "zero_copy_release_path"):
    for n in ("64", "512", "1024"):
        line = f"{leg:24s} {n:>5s}"
        for t in ("prod", "noacq"):
            v = sorted(r[leg][n]["service_us"] for r in rows[t])
            line += f"  {t} {statistics.median(v):6.2f} [{v[0]:.2f}-{v[-1]:.2f}]"
        print(line)
P
