#!/bin/bash
# Round 5, second GPU session: the PMC refresh of every product workload (profiles/pmc_traffic.json, with kernel code
# hashes), the uncached-ring experiment and the TX variants under the same passes; then the TX phase split A/B.
#   bash scripts/gpu_r5_b.sh <tag>
set -o pipefail
TAG=${1:-r5pmc}
bash scripts/pmc_refresh.sh $TAG "--uncached --tx-variants 40,51,52,13,14" || exit $?
mkdir -p gpurun_out/$TAG
for off in 14 2; do
  timeout -k 10 300 python scripts/tx_variants.py --frame-off $off --variants 40,13,14,9,51 --rotate 4 --rounds 9 \
    > gpurun_out/$TAG/tx_split_off$off.out 2> gpurun_out/$TAG/tx_split_off$off.err
  rc=$?; echo "tx_split_off$off rc=$rc"
  case $rc in 0|1) ;; *) exit $rc ;; esac
done
