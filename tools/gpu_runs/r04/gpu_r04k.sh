# r04k: output-path and chain tests (IPOutputCombo's verdict-carried
# rewrite), the glue fault tests, the adapter core, then config 1
set -o pipefail
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_chain.py tests/test_gpu_output_elements.py tests/test_gpu_adapter_core.py tests/test_gpu_glue_faults.py tests/test_gpu_elements.py > $O/tests.log 2>&1 || exit 2
timeout -k 10 600 python -u -c "
import json, click_amd, bench, torch
ctx = click_amd.Context(0)
bench.load_torch_kernels(torch)
print(json.dumps(bench.config1(ctx)))
" > $O/c1.json 2> $O/c1.err || exit 4
