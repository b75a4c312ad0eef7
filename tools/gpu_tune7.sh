set -o pipefail
mkdir -p gpurun_out
TUNE_ELEMENT=CheckUDPHeader timeout -k 10 200 python tools/tune.py --workload c4 --variants base,smark,smark_kv4 --rounds 6 > gpurun_out/t_c4c.json 2>gpurun_out/t.err || exit 2
TUNE_ELEMENT=SetUDPChecksum timeout -k 10 200 python tools/tune.py --workload c4 --variants base,smark --rounds 6 > gpurun_out/t_c4s.json 2>>gpurun_out/t.err || exit 3
