set -o pipefail
mkdir -p gpurun_out/sp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/sp/gpu_all.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/sp/bench.json 2>gpurun_out/sp/bench.err || exit 2
