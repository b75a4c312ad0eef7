#!/bin/bash
# r03k: glue tests (header-only staging), C4 packet-stream grid caps (waves
# taking several runs, so the next run's descriptors load ahead) for Check
# and Set, dense Set variants, then the default bench (oracle digest after
# the timed regions)
O=gpurun_out/r03k; mkdir -p $O
. tools/gpu_step.sh
step glue timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_elements.py tests/test_gpu_glue_faults.py tests/test_gpu_zerocopy.py tests/test_gpu_output.py tests/test_gpu_output_elements.py > $O/gpu_glue_tests.log 2>&1
step c4check env TUNE_ELEMENT=CheckUDPHeader timeout -k 10 300 python tools/tune.py --workload c4 --variants base,mb1280,mb2560,mb4k,mb8k,mb16k,mb64k --rounds 6 > $O/tune_c4_check.json 2> $O/tune_c4_check.err
step c4set env TUNE_ELEMENT=SetUDPChecksum timeout -k 10 300 python tools/tune.py --workload c4 --variants base,dset,dsetk3,dsetk4,mb2560,mb8k,mb32k --rounds 5 > $O/tune_c4_set.json 2> $O/tune_c4_set.err
step bench timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
