#!/bin/bash
# r03z: the RCCL code path of bench.py with one rank (and the gloo two-rank rehearsal)
O=gpurun_out/r03z; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bench_sizes.py -k "rccl or two_ranks" > $O/gpu_tests.log 2>&1
