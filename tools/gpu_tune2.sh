set -o pipefail
mkdir -p gpurun_out
TUNE_ELEMENT=CheckUDPHeader timeout -k 10 200 python tools/tune.py --workload c3 --variants base,nt,k4,k12,k16,g8 > gpurun_out/t_c3c.json 2>gpurun_out/t.err || exit 1
TUNE_ELEMENT=CheckUDPHeader timeout -k 10 200 python tools/tune.py --workload c4 --variants base,nt > gpurun_out/t_c4c.json 2>>gpurun_out/t.err || exit 2
TUNE_ELEMENT=SetUDPChecksum timeout -k 10 200 python tools/tune.py --workload c4 --variants base,fused_stream > gpurun_out/t_c4s.json 2>>gpurun_out/t.err || exit 3
TUNE_ELEMENT=SetUDPChecksum timeout -k 10 200 python tools/tune.py --workload c3 --variants base,fused,nt > gpurun_out/t_c3s.json 2>>gpurun_out/t.err || exit 4
