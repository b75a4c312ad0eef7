set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "size_class" --timeout 120 --timeout-method thread > gpurun_out/t_varlen.log 2>&1 || exit 1
TUNE_ELEMENT=CheckUDPHeader timeout -k 10 240 python tools/tune.py --workload c4 --variants range,stream,skv1,skv4,skv8 > gpurun_out/tune_c4_check.json 2> gpurun_out/tune_c4_check.err || exit 2
TUNE_ELEMENT=SetUDPChecksum timeout -k 10 240 python tools/tune.py --workload c4 --variants range,stream,skv4 > gpurun_out/tune_c4_set.json 2> gpurun_out/tune_c4_set.err || exit 3
