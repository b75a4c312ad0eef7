# r05u: the threaded glue, ZEROCOPY and staged, with the kernels' own time:
# does the ZEROCOPY Set stop scaling because its kernel writes the
# checksums into host memory over PCIe?
set -o pipefail
O=gpurun_out/r05u; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 tests/native/bin/mt_glue 4194304 "" zerocopy >> $O/mt.json 2>> $O/mt.err || exit 1
  timeout -k 10 300 tests/native/bin/mt_glue 4194304 "" staged >> $O/mt.json 2>> $O/mt.err || exit 2
done
echo ok >> $O/steps.txt
