#!/bin/bash
# chain_prof variants A/B, interleaved (tools/chain_prof/variants.sh)
set -o pipefail
O=$PWD/gpurun_out/r05y; mkdir -p $O
cd tools/chain_prof/bin
F=$(cat frame.hex)
for r in 1 2 3; do
  for v in ${VARIANTS:-chain_prof chain_prof_pf8 chain_prof_pf16 chain_prof_pf24 chain_prof_pf40}; do
    for c in elements combos; do
      echo -n "$v $c " >> $O/ab.txt
      timeout -k 10 60 ./$v $F 20 65536 $c > $O/one.json || exit 1
      python3 -c "import json,sys; d=json.load(open('$O/one.json')); print(d['mpps'], d['ns_per_packet'])" >> $O/ab.txt
    done
  done
done
