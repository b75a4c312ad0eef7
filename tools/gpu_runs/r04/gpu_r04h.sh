# r04h: chain + output-element + adapter-core tests, the pull-mode legs,
# then config-1 legs (elements one by one, chains at 64K and 16K batches,
# the zero-copy chain)
set -o pipefail
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_chain.py tests/test_gpu_output_elements.py tests/test_gpu_adapter_core.py > $O/tests.log 2>&1 || exit 2
timeout -k 10 300 tests/native/bin/pull_bench > $O/pull.json 2> $O/pull.err || exit 3
timeout -k 10 600 python -u -c "
import json, click_amd, bench, torch
ctx = click_amd.Context(0)
bench.load_torch_kernels(torch)
print(json.dumps(bench.config1(ctx)))
" > $O/c1.json 2> $O/c1.err || exit 4
