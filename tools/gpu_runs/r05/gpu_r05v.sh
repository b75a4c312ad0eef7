# r05v: as r05u, best of five runs, threads spread over the cores
# does the ZEROCOPY Set stop scaling because its kernel writes the
# checksums into host memory over PCIe?
set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
for r in 1; do
  timeout -k 10 300 tests/native/bin/mt_glue 4194304 "" zerocopy >> $O/mt.json 2>> $O/mt.err || exit 1
  timeout -k 10 300 tests/native/bin/mt_glue 4194304 "" staged >> $O/mt.json 2>> $O/mt.err || exit 2
done
echo ok >> $O/steps.txt
