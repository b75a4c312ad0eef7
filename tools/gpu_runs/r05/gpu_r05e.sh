# r05e: chains with IPOutputCombo after the head (clones from kept bytes),
# push retry after a failed chain flush; the core's tests; glue threads;
# read ceiling shape
set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 tests/native/bin/hipcore_test > $O/hipcore_test.log 2>&1
rc=$?; echo "hipcore_test rc=$rc" >> $O/steps.txt; [ $rc -le 1 ] || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_chain.py tests/test_gpu_adapter_core.py tests/test_gpu_output_elements.py tests/test_gpu_glue_faults.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/steps.txt; [ $rc -le 1 ] || exit 2
timeout -k 10 200 python -u -c "
import torch, click_amd, bench
ctx = click_amd.Context(0)
print('read_stream GB/s', bench.read_stream_peak(torch, ctx))
" > $O/read.txt 2>&1 || exit 3
echo "read ok" >> $O/steps.txt
