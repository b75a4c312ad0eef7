set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fragment.py tests/test_gpu_output_elements.py > gpurun_out/t_fragtest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c3 --no-c2 --skip c4,c5 --no-cpu > gpurun_out/b_c3.json 2>gpurun_out/b_c3.err || exit 2
