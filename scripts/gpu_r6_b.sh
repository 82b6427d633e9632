#!/bin/bash
# Round 6, second GPU session: the chain links (GPU pass vs the oracle) and the service tests, the whole GPU suite,
# the service's large-post sizing, the host A/B (merge + inline, and the chain links' in-order fast path), the bench.
# Each step has its own time limit; after an abort, a segfault or a time limit nothing more runs.
#   bash scripts/gpu_r6_b.sh <tag>
set -o pipefail
TAG=${1:-r6b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0|1) return 1 ;; *) return 0 ;; esac; }
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?
  echo "$name rc=$rc"
  if fatal $rc; then echo "stopping after $name (rc $rc)"; tail -30 $OUT/$name.out; exit $rc; fi
  return 0
}
step links 400 python -u -m pytest tests/test_gpu_links.py tests/test_gpu_service.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
tail -4 $OUT/links.out
step tests 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider
tail -4 $OUT/tests.out
step sizing 300 python scripts/service_sizing.py --waves 64,1088,2112,3136
cat $OUT/sizing.out
step host_ab 500 bash scripts/host_ab.sh $TAG/ab 4 scratch_ab/srv_B scratch_ab/srv_C
cat $OUT/host_ab.out
python3 - $OUT/ab <<'P'
import json, glob, sys, statistics
for f in ("srv_C",):
    d=[json.load(open(x)) for x in sorted(glob.glob(f"{sys.argv[1]}/{f}.pair.*.json"))]
    for k in ("gpu_rxbatch_512_pipelined_resident_release_path","gpu_rxbatch_512_pipelined_resident_unlinked_release_path","reference_server_release_build"):
        print(f, k, statistics.median(x[k]["mframes_per_s"] for x in d))
    t=[json.load(open(x)) for x in sorted(glob.glob(f"{sys.argv[1]}/{f}.twin.*.json"))]
    for k in ("cpu_rxbatch_512_pipelined_release_path_timed","cpu_rxbatch_512_pipelined_linked_release_path_timed"):
        print(f, k, statistics.median(x[k]["ns_per_frame_dispatch"] for x in t))
P
step bench 420 python bench.py
python3 -c "import json; L=json.load(open('$OUT/bench.out')); print(json.dumps(L['summary']))"
