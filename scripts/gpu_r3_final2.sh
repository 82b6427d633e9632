#!/bin/bash
# Round-3 final tree (after the window / pipelining / descriptor changes): parity suite + smoke, the default
# bench line, rocprofv3 kernel traces of the full bench and of the C2 line alone, and the C2 PMC passes.
#   bash scripts/gpu_r3_final2.sh <tag>      (C3/C5 PMC: bash scripts/gpu_pmc.sh <tag>/pmc_c3 3, ... 5)
set -o pipefail
TAG=${1:-r3final2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 \
  || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o trace -- \
  python3 bench.py --no-cpu-baseline --no-e2e --no-secondary --steps 50 > $OUT/prof_c2_bench.json 2> $OUT/prof_c2.err || { echo "c2 trace failed"; tail -20 $OUT/prof_c2.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_full -o trace -- \
  python3 bench.py --no-cpu-baseline --no-e2e --steps 50 > $OUT/prof_full_bench.json 2> $OUT/prof_full.err || { echo "full trace failed"; tail -20 $OUT/prof_full.err; exit 1; }
bash scripts/gpu_pmc.sh $TAG/pmc_c2 2 > $OUT/pmc_c2.log 2>&1 || { echo "pmc c2 failed"; tail -5 $OUT/pmc_c2.log; exit 1; }
echo final-ok
