set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
TUNE_ELEMENT=CheckUDPHeader timeout -k 10 200 python tools/tune.py --workload c3 --variants base,nont --rounds 8 > gpurun_out/t_c3c.json 2>gpurun_out/t.err || exit 2
TUNE_ELEMENT=CheckTCPHeader timeout -k 10 200 python tools/tune.py --workload c5 --variants base,nont --rounds 4 > gpurun_out/t_c5c.json 2>>gpurun_out/t.err || exit 3
TUNE_ELEMENT=SetUDPChecksum timeout -k 10 200 python tools/tune.py --workload c4 --variants base,two_stream > gpurun_out/t_c4s.json 2>>gpurun_out/t.err || exit 4
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 5
