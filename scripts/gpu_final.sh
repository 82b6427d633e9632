#!/bin/bash
# End-of-session GPU pass: parity suite + smoke, the C2 bench line with its rocprofv3 kernel
# stats, C3/C5 bench lines, and the PMC traffic passes (scripts/gpu_pmc.sh) for C2/C3/C5.
#   bash scripts/gpu_final.sh <tag>
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash scripts/gpu_check.sh $TAG > $OUT/check.log 2>&1 || { tail -20 $OUT/check.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
for c in 3 5; do
  timeout -k 10 300 python bench.py --config $c --no-e2e --cpu-seconds 4 > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err || { tail $OUT/bench_c$c.err; exit 1; }
done
for c in 2 3 5; do
  bash scripts/gpu_pmc.sh ${TAG}_pmc_c$c $c > /dev/null 2>&1 || { echo "pmc c$c failed"; exit 1; }
done
echo final-ok
