#!/bin/bash
# PC-sampled combos: chain vs separate elements, staged and ZEROCOPY
set -o pipefail
O=$PWD/gpurun_out/r05ad; mkdir -p $O
for mode in zerocopy staged; do
  for sep in chain separate; do
    RUNS=30 CHAIN=combos MODE=$mode SEP=$sep SAMPLES=$O/combos_${mode}_$sep.samples timeout -k 10 120 bash tools/chain_prof/run.sh run > $O/combos_${mode}_$sep.txt 2>&1 || exit 1
    RUNS=30 CHAIN=combos MODE=$mode SEP=$sep timeout -k 10 120 bash tools/chain_prof/run.sh run > $O/combos_${mode}_${sep}_nosample.txt 2>&1 || exit 1
  done
done
