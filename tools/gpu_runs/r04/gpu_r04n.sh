# r04n: the chunked two-phase Set (set_chunks): parity, then an interleaved
# A/B of 1 / 2 / 4 / 8 / 16 ranges on C3 SetUDPChecksum and C5 SetTCPChecksum
set -o pipefail
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "chunked or set_modes" > $O/tests.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/tune.py --workload c3 --variants base,ch2,ch4,ch8,ch16 --rounds 6 > $O/tune_c3.json 2> $O/tune_c3.err || exit 3
timeout -k 10 400 python -u tools/tune.py --workload c5 --variants base,ch4,ch8,ch16 --rounds 4 --launches 3 > $O/tune_c5.json 2> $O/tune_c5.err || exit 4
