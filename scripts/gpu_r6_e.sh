#!/bin/bash
# Round 6: the drop-in server pipelined one vs two polls deep (Conf::RxPipelineDepth) -- the peer parity test on
# the GPU (every RX mode, depth 2 included, equal to the twin), then the depth A/B beside the reference's server with
# the host's wait per poll timed, rounds interleaved.   bash scripts/gpu_r6_e.sh <tag>
set -o pipefail
TAG=${1:-r6e2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
fatal() { case $1 in 0|1) return 1 ;; *) return 0 ;; esac; }
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?
  echo "$name rc=$rc"
  if fatal $rc; then echo "stopping after $name (rc $rc)"; tail -30 $OUT/$name.out; exit $rc; fi
  return 0
}
step peer 400 ./tests/cpp/test_tcp_server_peer gpu
grep -E "^\[|gpu: handler|FAIL|PASS" $OUT/peer.out | tail -20
for r in 1 2 3 4 5; do
  step depth.$r 120 ./bench/bench_tcp_server 256 3000 depth_ab
done
python3 - $OUT <<'P'
import json, glob, sys, statistics
rows = [json.load(open(f)) for f in sorted(glob.glob(f"{sys.argv[1]}/depth.*.out"))]
keys = ["gpu_rxbatch_512_pipelined_resident_release_path_timed", "gpu_rxbatch_512_pipelined2_resident_release_path_timed",
        "gpu_rxbatch_512_pipelined2_resident_release_path", "reference_server_release_build"]
for k in keys:
    v = [r[k] for r in rows if k in r and "mframes_per_s" in r[k]]
    if not v: continue
    m = [x["mframes_per_s"] for x in v]; so = [x["mframes_per_s_server_only"] for x in v]
    w = [x.get("wait_us_per_poll", -1) for x in v]
    print(f"{k:58s} Mfps {statistics.median(m):6.2f} [{min(m):.2f}-{max(m):.2f}] server-only {statistics.median(so):6.2f} wait us/poll {statistics.median(w):.3f}")
P
