# r04g: element chains (clk_chain_*) against the elements one by one; the
# config-1 bench legs with chains; the native adapter test
set -o pipefail
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_chain.py tests/test_gpu_adapter_core.py > $O/tests.log 2>&1
echo "tests rc=$?" >> $O/steps.txt
timeout -k 10 600 python -u -c "
import json, click_amd, bench, torch
ctx = click_amd.Context(0)
bench.load_torch_kernels(torch)
print(json.dumps(bench.config1(ctx)))
" > $O/c1.json 2> $O/c1.err || exit 3
