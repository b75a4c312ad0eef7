# r05l: chains as per-member lists (prep / route loops), IPOutputCombo after
# the head, push retry; core tests; config 1 legs; read ceiling shapes;
# threaded glue
set -o pipefail
O=gpurun_out/r05l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 tests/native/bin/hipcore_test > $O/hipcore_test.log 2>&1
rc=$?; echo "hipcore_test rc=$rc" >> $O/steps.txt; [ $rc -le 1 ] || exit 1
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_chain.py tests/test_gpu_adapter_core.py tests/test_gpu_output_elements.py tests/test_gpu_glue_faults.py tests/test_gpu_zerocopy.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/steps.txt; [ $rc -le 1 ] || exit 2
timeout -k 10 600 python -u -c "
import json, click_amd, bench, torch
ctx = click_amd.Context(0)
bench.load_torch_kernels(torch)
d = {}
print(json.dumps({'read': bench.read_stream_peak(torch, ctx, detail=d), 'shapes': d}))
print(json.dumps(bench.config1(ctx)))
" > $O/c1.json 2> $O/c1.err || exit 3
echo "c1 ok" >> $O/steps.txt
timeout -k 10 300 tests/native/bin/pull_bench > $O/pull.json 2> $O/pull.err || exit 4
echo "pull ok" >> $O/steps.txt
