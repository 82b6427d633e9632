#!/bin/bash
# Round 6: the service with its mailbox in device memory, read by every wave (no wave-0 hand-off).  The service,
# link and server GPU tests first; then interleaved A/B rounds against the previous protocol (ab_libs/old, the same
# sources with the round-5 rx_service.hip; LD_LIBRARY_PATH picks it): post round trips (bench_signal) and the
# drop-in server pair (bench_tcp_server resident_pair).   bash scripts/gpu_r6_m.sh <tag>
set -o pipefail
TAG=${1:-r6m}
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
step tests 400 python -u -m pytest tests/test_gpu_service.py tests/test_gpu_links.py tests/test_tcp_server.py tests/test_ref_conn.py -m gpu -x -v \
  --timeout 200 --timeout-method thread -p no:cacheprovider
tail -3 $OUT/tests.out
grep -q " passed" $OUT/tests.out && ! grep -q -E "FAILED|ERROR" $OUT/tests.out || { grep -E "FAILED|ERROR|Error" $OUT/tests.out | head -20; exit 1; }
for r in 1 2 3; do
  step sig_new.$r 120 ./bench/bench_signal 400
  LD_LIBRARY_PATH=$PWD/ab_libs/old step sig_old.$r 120 ./bench/bench_signal 400
done
for r in 1 2 3; do
  step pair_new.$r 120 ./bench/bench_tcp_server 256 3000 resident_pair
  LD_LIBRARY_PATH=$PWD/ab_libs/old step pair_old.$r 120 ./bench/bench_tcp_server 256 3000 resident_pair
done
python3 - $OUT <<'P'
import json, glob, sys, statistics
o = sys.argv[1]
def load(pat): return [json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob(f"{o}/{pat}"))]
for tag in ("new", "old"):
    rows = load(f"sig_{tag}.*.out")
    for leg in ("resident", "zero_copy", "resident_release_path", "zero_copy_release_path"):
        for n in ("64", "512", "1024"):
            v = [r[leg][n]["service_us"] for r in rows]
            print(tag, leg, n, "service_us", [round(x, 2) for x in v], "records_equal", all(r[leg][n]["records_equal"] for r in rows))
for tag in ("new", "old"):
    rows = load(f"pair_{tag}.*.out")
    g = [r["gpu_rxbatch_512_pipelined_resident_release_path"]["mframes_per_s"] for r in rows]
    ref = [r["reference_server_release_build"]["mframes_per_s"] for r in rows]
    print(tag, "pair gpu", g, "reference", ref)
P
