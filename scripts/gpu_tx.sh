#!/bin/bash
# TX checksum fill session: TX GPU tests, the A/B variants, bench_tx, kernel trace of bench_tx.
# Usage (repo root, GPU box): bash scripts/gpu_tx.sh <tag>
set -o pipefail
TAG=${1:-tx}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tx.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tx_tests.log 2>&1
RC=$?; echo "tx pytest rc=$RC"; tail -4 $OUT/tx_tests.log
[ $RC -eq 0 ] || exit $RC
timeout -k 10 300 python scripts/tx_variants.py --frame-off 2 > $OUT/variants_off2.json 2> $OUT/variants.err || { echo "variants failed"; tail $OUT/variants.err; exit 1; }
timeout -k 10 300 python scripts/tx_variants.py --frame-off 14 > $OUT/variants_off14.json 2>> $OUT/variants.err || { echo "variants failed"; tail $OUT/variants.err; exit 1; }
python -c "
import json
for f in ('off2','off14'):
    d=json.load(open('$OUT/variants_'+f+'.json')); print(f, {k:v['ms_median'] for k,v in d.items() if isinstance(v,dict)})"
timeout -k 10 300 python scripts/bench_tx.py > $OUT/bench_tx.json 2> $OUT/bench_tx.err || { echo "bench_tx failed"; tail $OUT/bench_tx.err; exit 1; }
cat $OUT/bench_tx.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o trace -- \
  python3 scripts/bench_tx.py --no-cpu-baseline --steps 30 > $OUT/prof_bench_tx.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \;
