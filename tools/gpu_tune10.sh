set -o pipefail
mkdir -p gpurun_out/sp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fragment.py tests/test_gpu_output_elements.py tests/test_gpu_zerocopy.py > gpurun_out/sp/frag.log 2>&1 || exit 1
TUNE_ELEMENT=IPFragmenter timeout -k 10 240 python tools/tune.py --workload c3 --variants base,fpro0 --rounds 8 --launches 3 > gpurun_out/sp/fr.json 2>gpurun_out/sp/fr.err || exit 2
timeout -k 10 300 python bench.py --workload c3 --no-c2 --skip c4,c5 --no-cpu > gpurun_out/sp/b_c3.json 2>gpurun_out/sp/b_c3.err || exit 3
