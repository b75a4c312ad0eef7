set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "run_" > gpurun_out/t.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
