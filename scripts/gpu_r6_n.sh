#!/bin/bash
# Round 6: the device-memory mailbox, post written as one 64-B non-temporal line (C, the product) vs two fenced
# stores (B, ab_libs/b) vs the round-5 protocol (A, ab_libs/old): the service tests on C, then bench_signal in five
# interleaved rounds of A, B, C.   bash scripts/gpu_r6_n.sh <tag>
set -o pipefail
TAG=${1:-r6n}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0|1) return 1 ;; *) return 0 ;; esac; }
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?
  echo "$name rc=$rc"
  if fatal $rc; then echo "stopping after $name (rc $rc)"; tail -30 $OUT/$name.out $OUT/$name.err; exit $rc; fi
  return 0
}
step tests 300 python -u -m pytest tests/test_gpu_service.py tests/test_gpu_links.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider
tail -2 $OUT/tests.out
grep -q " passed" $OUT/tests.out && ! grep -q -E "FAILED|ERROR" $OUT/tests.out || { grep -E "FAILED|ERROR|Error" $OUT/tests.out | head -20; exit 1; }
for r in 1 2 3 4 5; do
  LD_LIBRARY_PATH=$PWD/ab_libs/old step sig_A.$r 120 ./bench/bench_signal 600
  LD_LIBRARY_PATH=$PWD/ab_libs/b step sig_B.$r 120 ./bench/bench_signal 600
  step sig_C.$r 120 ./bench/bench_signal 600
done
python3 - $OUT <<'P'
import json, glob, sys, statistics
o = sys.argv[1]
def load(pat): return [json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob(f"{o}/{pat}"))]
rows = {t: load(f"sig_{t}.*.out") for t in "ABC"}
for leg in ("resident", "zero_copy", "resident_release_path", "zero_copy_release_path"):
    for n in ("64", "512", "1024"):
        line = f"{leg:24s} {n:>5s}"
        for t in "ABC":
            v = sorted(r[leg][n]["service_us"] for r in rows[t])
            line += f"  {t} {statistics.median(v):6.2f} [{v[0]:.2f}-{v[-1]:.2f}]"
        ok = all(r[leg][n]["records_equal"] for t in "ABC" for r in rows[t])
        print(line, "records_equal" if ok else "RECORDS DIFFER")
P
