#!/bin/bash
# r03l (2nd try): stream parity with the default library (phase A as at
# HEAD), then the same tests with the two-deep dense variant swapped in,
# then C4 Check variants; stops at the first failure
O=gpurun_out/r03l; mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $PT tests/test_gpu_parity.py tests/test_gpu_bench_sizes.py > $O/gpu_tests.log 2>&1 || exit 1
cp click_amd/libclick_amd_cksum.so /tmp/lib_base.so && cp build/variants/lib_dd2.so click_amd/libclick_amd_cksum.so || exit 2
timeout -k 10 600 $PT tests/test_gpu_parity.py -k "variable_length or stream or fuzz or golden or run_tails" > $O/gpu_tests_dd2.log 2>&1
rc=$?; cp /tmp/lib_base.so click_amd/libclick_amd_cksum.so; [ $rc -eq 0 ] || exit 3
TUNE_ELEMENT=CheckUDPHeader timeout -k 10 300 python tools/tune.py --workload c4 --variants prev,base,dd2,dd2k3w6,dd2k2w8 --rounds 8 > $O/tune_c4_check.json 2> $O/tune_c4_check.err
