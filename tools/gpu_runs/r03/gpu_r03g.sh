#!/bin/bash
# r03g: dense run-ahead without stray waits: parity + C4 Check variants
O=gpurun_out/r03g; mkdir -p $O
. tools/gpu_step.sh
step tests timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_bench_sizes.py > $O/gpu_tests.log 2>&1
step c4check env TUNE_ELEMENT=CheckUDPHeader timeout -k 10 300 python tools/tune.py --workload c4 --variants base,dense0,dk4,dk4w4,ahead0 --rounds 6 > $O/tune_c4_check.json 2> $O/tune_c4_check.err
