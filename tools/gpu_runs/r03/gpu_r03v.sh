#!/bin/bash
# r03v: empty batches and maximum IP length through every path
O=gpurun_out/r03v; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "empty or maximum" > $O/gpu_tests.log 2>&1
