set -o pipefail
mkdir -p gpurun_out
TUNE_ELEMENT=CheckUDPHeader timeout -k 10 200 python tools/tune.py --workload c4 --variants base,hc2,hc2w8,w8 --rounds 6 > gpurun_out/t_c4c.json 2>gpurun_out/t.err || exit 2
TUNE_ELEMENT=SetUDPChecksum timeout -k 10 200 python tools/tune.py --workload c4 --variants base,hc2w8 --rounds 6 > gpurun_out/t_c4s.json 2>>gpurun_out/t.err || exit 3
