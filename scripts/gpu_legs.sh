#!/bin/bash
# Clean rocprof pair for the C2 bench kernel (no secondary workloads in the traced run), the
# drop-in server's per-poll HIP API costs (hip + kernel trace of bench_tcp_server quick), and
# the zero-copy classify leg on its own (bench_pinned), all on one box.
#   bash scripts/gpu_legs.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-legs}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o trace -- \
  python3 bench.py --no-cpu-baseline --no-e2e --no-secondary --steps 50 > $OUT/prof_bench.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
timeout -k 10 180 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $OUT/srv -o srv -- \
  ./bench/bench_tcp_server 256 400 quick > $OUT/srv.json 2> $OUT/srv.err || { tail -20 $OUT/srv.err; exit 1; }
timeout -k 10 120 ./bench/bench_pinned 200 > $OUT/pinned.json 2> $OUT/pinned.err || { tail -20 $OUT/pinned.err; exit 1; }
echo legs-ok
