#!/bin/bash
# chain_prof variants A/B, interleaved: VARIANTS, CHAINS, MODES, SEPS, ROUNDS; output $OUT/ab.txt
set -o pipefail
O=$PWD/gpurun_out/${OUT:-ab}; mkdir -p $O; rm -f $O/ab.txt
cd tools/chain_prof/bin
F=$(cat frame.hex)
for r in $(seq ${ROUNDS:-3}); do
  for v in $VARIANTS; do
    for c in ${CHAINS:-combos elements}; do
      for m in ${MODES:-staged zerocopy}; do
        for s in ${SEPS:-chain}; do
          timeout -k 10 60 ./$v $F ${RUNS:-20} 65536 $c $m $s > $O/one.json || exit 1
          python3 -c "import json; d=json.load(open('$O/one.json')); print('$v', d['leg'], d['mpps'])" >> $O/ab.txt
        done
      done
    done
  done
done
