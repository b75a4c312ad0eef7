#!/bin/bash
# streaming-store staging: glue tests + e2e
set -o pipefail
O=$PWD/gpurun_out/r05ac; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_chain.py tests/test_gpu_elements.py tests/test_gpu_output_elements.py tests/test_gpu_adapter_core.py tests/test_gpu_glue_faults.py tests/test_gpu_threads.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 900 python bench.py --e2e > $O/e2e.json 2> $O/e2e.err || exit 3
