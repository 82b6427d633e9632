#!/bin/bash
# One GPU session: parity tests, bench line, rocprofv3 kernel-trace stats.
# Usage (from the repo root, on the GPU box): bash scripts/gpu_check.sh <tag>
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
RC=$?
echo "pytest rc=$RC" | tee -a $OUT/gpu_tests.log
[ $RC -le 1 ] || { tail -30 $OUT/gpu_tests.log; exit $RC; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o trace -- \
  python3 bench.py --no-cpu-baseline --no-e2e --no-secondary --steps 50 > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \;
