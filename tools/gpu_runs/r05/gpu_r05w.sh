#!/bin/bash
# line-level gprof of the combos and element chains (tools/chain_prof)
set -o pipefail
O=gpurun_out/r05w; mkdir -p $O
RUNS=40 CHAIN=combos TOPL=90 timeout -k 10 240 bash tools/chain_prof/run.sh run > $O/combos.txt 2>&1 &&
RUNS=40 CHAIN=elements TOPL=90 timeout -k 10 240 bash tools/chain_prof/run.sh run > $O/elements.txt 2>&1
