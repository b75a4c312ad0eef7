# r05n: chain host cost against the batch size (tools/chain_prof, no gprof
# output needed: its JSON line carries ns per packet by phase)
set -o pipefail
O=gpurun_out/r05n; mkdir -p $O
cd tools/chain_prof/bin
for c in elements combos; do for b in 4096 8192 16384 32768 65536; do
  timeout -k 10 60 ./chain_prof $(cat frame.hex) 20 $b $c | sed "s/^{/{\"batch\": $b, /" >> ../../../$O/batch.json || exit 1
done; done
echo ok >> ../../../$O/steps.txt
