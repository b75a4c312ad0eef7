# r04c: glue fault tests (ZEROCOPY abandon at every step), high-address
# parity, then the split readfirstlane variants under the address check
# (risky step last; it stops at the first variant that faults)
set -o pipefail
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_glue_faults.py tests/test_gpu_parity.py -k "zerocopy or high_address or variable_length" > $O/tests.log 2>&1 || exit 11
timeout -k 10 900 python -u tools/addr_check/addr_check.py run $O/addr_check.json sgpr_u32,total_only,base_int_only,sgpr_int > $O/addr_check.log 2>&1 || exit 13
