# r04a: root-cause run of round 3's stream-kernel fault (address-checked
# libraries), the high-address parity test, and the fragmenter fused /
# unfused / XCD-ordered A/B
set -o pipefail
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 900 python -u tools/addr_check/addr_check.py run $O/addr_check.json > $O/addr_check.log 2>&1 || exit 11
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "variable_length or high_address or dense_and_generic" > $O/parity.log 2>&1 || exit 12
TUNE_ELEMENT=IPFragmenter timeout -k 10 600 python -u tools/tune.py --workload c3 --variants base,ffu0,ffu0xcd --rounds 8 --launches 5 > $O/tune_frag.json 2> $O/tune_frag.err || exit 13
