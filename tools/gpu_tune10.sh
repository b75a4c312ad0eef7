set -o pipefail
mkdir -p gpurun_out/sp
TUNE_ELEMENT=SetUDPChecksum timeout -k 10 200 python tools/tune.py --workload c3 --variants base,fused,fusednt --rounds 6 --launches 3 > gpurun_out/sp/s3.json 2>gpurun_out/sp/s.err || exit 3
TUNE_ELEMENT=SetTCPChecksum timeout -k 10 300 python tools/tune.py --workload c5 --variants base,fused,fusednt --rounds 3 --launches 2 > gpurun_out/sp/s5.json 2>>gpurun_out/sp/s.err || exit 2
