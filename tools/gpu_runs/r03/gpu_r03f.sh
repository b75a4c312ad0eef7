#!/bin/bash
# r03f: dense runs with the next run's first pass issued ahead: parity, C4
# Check / Set variants, glue tests (16 B staging slots, shared chatter), c1
O=gpurun_out/r03f; mkdir -p $O
. tools/gpu_step.sh
step tests timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_bench_sizes.py > $O/gpu_tests.log 2>&1
step c4check env TUNE_ELEMENT=CheckUDPHeader timeout -k 10 300 python tools/tune.py --workload c4 --variants base,dense0,dk4,dk4w4,ahead0 --rounds 6 > $O/tune_c4_check.json 2> $O/tune_c4_check.err
step c4set env TUNE_ELEMENT=SetUDPChecksum timeout -k 10 300 python tools/tune.py --workload c4 --variants base,dset --rounds 6 > $O/tune_c4_set.json 2> $O/tune_c4_set.err
step glue timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_elements.py tests/test_gpu_glue_faults.py tests/test_gpu_zerocopy.py tests/test_gpu_adapter_core.py tests/test_gpu_output_elements.py > $O/gpu_glue_tests.log 2>&1
step c1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --workload c2 --no-cpu --no-peak --skip c4,c5 --no-verify > $O/bench_c1.json 2> $O/bench_c1.err
