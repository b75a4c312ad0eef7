# r04b: default bench (summary / comm keys), C3 profile with the fragmenter
# (FETCH/WRITE counters of frag_write_kernel), then the split readfirstlane
# variants under the address check (the risky step last; it stops at the
# first variant that faults)
set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 11
FRAG=1 timeout -k 10 900 bash tools/profile.sh r04 c3 || exit 12
timeout -k 10 900 python -u tools/addr_check/addr_check.py run $O/addr_check.json sgpr_u32,total_only,base_int_only,sgpr_int > $O/addr_check.log 2>&1 || exit 13
