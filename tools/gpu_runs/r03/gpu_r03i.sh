#!/bin/bash
# r03i: stream kernel without the tail stash (end-masked last chunks, 6
# waves): parity (incl. padded packets), C4 Check / Set variants
O=gpurun_out/r03i; mkdir -p $O
. tools/gpu_step.sh
step tests timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_bench_sizes.py tests/test_gpu_elements.py > $O/gpu_tests.log 2>&1
step c4check env TUNE_ELEMENT=CheckUDPHeader timeout -k 10 300 python tools/tune.py --workload c4 --variants base,dense0,dk4,dk6w4 --rounds 6 > $O/tune_c4_check.json 2> $O/tune_c4_check.err
step c4set env TUNE_ELEMENT=SetUDPChecksum timeout -k 10 300 python tools/tune.py --workload c4 --variants base,dset --rounds 5 > $O/tune_c4_set.json 2> $O/tune_c4_set.err
