set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
TUNE_ELEMENT=CheckIPHeader timeout -k 10 200 python tools/tune.py --workload c2 --variants base,nont --rounds 8 > gpurun_out/t_c2c.json 2>gpurun_out/t.err || exit 2
timeout -k 10 300 python bench.py --no-c2 --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 5
