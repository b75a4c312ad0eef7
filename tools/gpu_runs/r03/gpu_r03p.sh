#!/bin/bash
# r03p: parity after removing the measured-slower knobs (stream + fixed geometry)
O=gpurun_out/r03p; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_bench_sizes.py > $O/gpu_tests.log 2>&1
