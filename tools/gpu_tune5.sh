set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_zerocopy.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
TUNE_ELEMENT=SetUDPChecksum timeout -k 10 200 python tools/tune.py --workload c3 --variants base,fused,fused_noblock --rounds 6 > gpurun_out/t_c3s.json 2>gpurun_out/t.err || exit 2
TUNE_ELEMENT=SetUDPChecksum timeout -k 10 200 python tools/tune.py --workload c4 --variants base,noblock,two_stream --rounds 6 > gpurun_out/t_c4s.json 2>>gpurun_out/t.err || exit 3
TUNE_ELEMENT=SetTCPChecksum timeout -k 10 300 python tools/tune.py --workload c5 --variants base,fused --rounds 3 > gpurun_out/t_c5s.json 2>>gpurun_out/t.err || exit 4
