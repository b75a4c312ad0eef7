#!/bin/bash
# r03w: the dense staging slots XOR-swizzled (LDS bank conflicts): parity
# with the variant swapped in, then C4 Check timing
O=gpurun_out/r03w; mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
cp click_amd/libclick_amd_cksum.so /tmp/lib_base.so && cp build/variants/lib_swz.so click_amd/libclick_amd_cksum.so || exit 2
timeout -k 10 600 $PT tests/test_gpu_parity.py -k "variable_length or stream or maximum or empty" > $O/gpu_tests_swz.log 2>&1
rc=$?; cp /tmp/lib_base.so click_amd/libclick_amd_cksum.so; [ $rc -eq 0 ] || exit 3
TUNE_ELEMENT=CheckUDPHeader timeout -k 10 300 python tools/tune.py --workload c4 --variants base,swz --rounds 10 > $O/tune_c4_check.json 2> $O/tune_c4_check.err
