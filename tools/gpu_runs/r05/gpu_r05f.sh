# r05f: chain tests after the clone / push-retry changes; the read ceiling
# over the probe's shapes; the threaded glue
set -o pipefail
O=gpurun_out/r05f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_chain.py tests/test_gpu_adapter_core.py tests/test_gpu_output_elements.py tests/test_gpu_glue_faults.py tests/test_gpu_zerocopy.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/steps.txt; [ $rc -le 1 ] || exit 2
timeout -k 10 200 python -u -c "
import torch, click_amd, bench
ctx = click_amd.Context(0)
d = {}
print('read_stream GB/s', bench.read_stream_peak(torch, ctx, detail=d), d)
" > $O/read.txt 2>&1 || exit 3
echo "read ok" >> $O/steps.txt
timeout -k 10 300 tests/native/bin/mt_glue > $O/mt.json 2> $O/mt.err || exit 4
echo "mt ok" >> $O/steps.txt
