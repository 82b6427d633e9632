#!/bin/bash
# Round 6, first GPU session: the resident-service tests first (the conn-table contract, the post limit, large posts
# on helper waves), then the whole GPU suite, then the default bench line (service sizing, the same-buffer TX pair,
# the hot / L3 / DRAM server pairs).  Each step has its own time limit; after an abort, a segfault or a time limit
# nothing more runs (an ordinary test failure, rc 1, does not stop the bench).   bash scripts/gpu_r6_a.sh <tag>
set -o pipefail
TAG=${1:-r6a}
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
step service 400 python -u -m pytest tests/test_gpu_links.py tests/test_gpu_service.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
tail -25 $OUT/service.out
step tests 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
tail -3 $OUT/tests.out
step bench 420 python bench.py
python3 -c "import json; L=json.load(open('$OUT/bench.out')); print(json.dumps(L['summary'])); print(json.dumps(L['secondary'].get('service_large_post')))"
# where the host spends a poll (item 2): the sampler (bench/sampler.hpp) over the best GPU leg, the reference's own
# server and the CPU twin's dispatch, on this box's cores; symbolized here (llvm-symbolizer) into text
{ cat /proc/sys/kernel/perf_event_paranoid; which perf; lscpu | grep -E "Model name|L3|L2"; } > $OUT/host_cpu.txt 2>&1
PN_SAMPLE=$OUT/samp step sample_pair 120 ./bench/bench_tcp_server 256 4000 resident_pair
PN_SAMPLE=$OUT/samp step sample_twin 120 ./bench/bench_tcp_server 256 4000 twin_timed
for t in gpu reference twin; do
  python3 scripts/sample_report.py bench/bench_tcp_server $OUT/samp.$t --top 45 --lines > $OUT/profile_$t.txt 2>&1
done
head -40 $OUT/profile_gpu.txt
step host_ab 400 bash scripts/host_ab.sh $TAG/ab 4 scratch_ab/srv_base scratch_ab/srv_A scratch_ab/srv_B
cat $OUT/host_ab.out
