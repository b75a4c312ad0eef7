# r04t: the pipelined fragmenter write loop (CLK_FRAG_PIPE): every -m gpu
# test, then the A/B against the serial loop (fpipe0) and the pipelined
# loop squeezed to 4 waves per SIMD (fpipew4)
set -o pipefail
O=gpurun_out/r04t; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || exit 1
echo "tests ok" >> $O/steps.txt
TUNE_ELEMENT=IPFragmenter timeout -k 10 600 python -u tools/tune.py --workload c3 --variants base,fpipe0,fpipew4 --rounds 8 --launches 5 > $O/tune_frag.json 2> $O/tune_frag.err || exit 2
echo "tune ok" >> $O/steps.txt
