#!/bin/bash
# inlined glue loops + push fast path: chain tests, glue tests, core tests, chain A/B
set -o pipefail
O=$PWD/gpurun_out/r05z; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_chain.py tests/test_gpu_elements.py tests/test_gpu_output_elements.py tests/test_gpu_adapter_core.py tests/test_gpu_glue_faults.py tests/test_gpu_zerocopy.py > $O/tests.log 2>&1 || exit 1
VARIANTS="${AB:-chain_prof chain_prof_push}" bash tools/gpu_runs/r05/gpu_r05y.sh || exit 2
cp gpurun_out/r05y/ab.txt $O/ab.txt
