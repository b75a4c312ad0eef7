#!/bin/bash
# PC-sampled combos and element chains (tools/chain_prof; resolved on the CPU side)
set -o pipefail
O=$PWD/gpurun_out/r05x; mkdir -p $O
RUNS=40 CHAIN=combos SAMPLES=$O/combos.samples timeout -k 10 240 bash tools/chain_prof/run.sh run > $O/combos.txt 2>&1 &&
RUNS=40 CHAIN=elements SAMPLES=$O/elements.samples timeout -k 10 240 bash tools/chain_prof/run.sh run > $O/elements.txt 2>&1
