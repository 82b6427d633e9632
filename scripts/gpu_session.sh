#!/bin/bash
# One GPU session for the bench line: multi-rank tests, the default bench line (secondary
# workloads included), a --gpus 2 rehearsal, rocprofv3 kernel stats of the bench command.
#   bash scripts/gpu_session.sh <tag>
set -o pipefail
TAG=${1:-session}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_multi.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/multi.log 2>&1
RC=$?; tail -4 $OUT/multi.log; [ $RC -eq 0 ] || exit $RC
( time timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err ) 2> $OUT/bench.time || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
cat $OUT/bench.time
timeout -k 10 300 python bench.py --gpus 2 --no-cpu-baseline --no-e2e --no-secondary > $OUT/bench_n2.json 2> $OUT/bench_n2.err || { echo "bench n2 failed"; tail $OUT/bench_n2.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o trace -- \
  python3 bench.py --no-cpu-baseline --no-e2e --no-secondary > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \; > $OUT/kernel_stats.csv
head -12 $OUT/kernel_stats.csv
echo session-ok
