# Round-end check on the GPU box: every -m gpu test, smoke(), the default bench.
set -o pipefail
mkdir -p gpurun_out/check
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/check/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/check/smoke.log 2>&1 || exit 2
timeout -k 10 600 python bench.py > gpurun_out/check/bench.json 2> gpurun_out/check/bench.err || exit 3
