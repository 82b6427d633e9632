#!/bin/bash
# SQ counters (wave cycles, waits, instruction counts) of the production RX kernel beside its
# no-walk and no-probe ablations (scripts/variants.py, variants 1 / 43 / 11), C3 and C5; each
# counter set in its own rocprofv3 --pmc pass.   bash scripts/sq_probe_pmc.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-sq_pmc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_avail.txt 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"
for c in ${CONFIGS:-3 5}; do
  for p in 1 2; do
    eval CN=\$P$p
    timeout -s KILL 120 rocprofv3 --pmc $CN --output-format csv -d $OUT/c${c}_p$p -o pmc -- \
      python3 scripts/variants.py --config $c --variants ${VARIANTS:-1,43,11} --rounds 2 --reps 2 > $OUT/c${c}_p$p.json 2> $OUT/c${c}_p$p.err \
      || { echo "pass c$c p$p failed"; tail -5 $OUT/c${c}_p$p.err; exit 1; }
  done
done
echo sq-ok
