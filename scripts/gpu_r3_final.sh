#!/bin/bash
# Round-3 final-tree GPU pass: parity suite + smoke, the default bench line, a rocprofv3 kernel trace of
# the FULL bench (secondary kernels included: C3/C5/packed/TX/match_streams/ceilings), and the PMC
# traffic passes for C2/C3/C5 (scripts/gpu_pmc.sh).   bash scripts/gpu_r3_final.sh <tag>
set -o pipefail
TAG=${1:-r3final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 \
  || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o trace -- \
  python3 bench.py --no-cpu-baseline --no-e2e --steps 50 > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
for c in 2 3 5; do
  bash scripts/gpu_pmc.sh $TAG/pmc_c$c $c > $OUT/pmc_c$c.log 2>&1 || { echo "pmc c$c failed"; tail -5 $OUT/pmc_c$c.log; exit 1; }
done
echo final-ok
