#!/bin/bash
# r03r: CheckIPHeader with U packets per lane pair (loads issued together):
# parity with the default and with U = 4 swapped in, then C2 timing
O=gpurun_out/r03r; mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $PT tests/test_gpu_parity.py tests/test_gpu_elements.py > $O/gpu_tests.log 2>&1 || exit 1
cp click_amd/libclick_amd_cksum.so /tmp/lib_base.so && cp build/variants/lib_iphu4.so click_amd/libclick_amd_cksum.so || exit 2
timeout -k 10 600 $PT tests/test_gpu_parity.py -k "golden or fuzz or check_ip or full_size" > $O/gpu_tests_u4.log 2>&1
rc=$?; cp /tmp/lib_base.so click_amd/libclick_amd_cksum.so; [ $rc -eq 0 ] || exit 3
TUNE_ELEMENT=CheckIPHeader timeout -k 10 300 python tools/tune.py --workload c2 --variants prev,base,iphu2,iphu4 --rounds 10 --launches 20 > $O/tune_c2_check.json 2> $O/tune_c2_check.err
