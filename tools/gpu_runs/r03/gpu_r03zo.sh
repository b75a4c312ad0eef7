#!/bin/bash
# scatter-order probe; fused two-byte Set inside runs; C2 TCC request sizes
set -e
O=gpurun_out/r03zo
mkdir -p $O
timeout -k 10 120 tools/probes/order_probe > $O/order.json
timeout -k 10 240 python3 -u tools/tune.py --workload c3 --variants base,fusedrb0,fusedrb0nt,fusedrb0nts,occ4,fused > $O/tune_c3_set.json
TUNE_ELEMENT=CheckUDPHeader timeout -k 10 120 python3 -u tools/tune.py --workload c3 --variants base > $O/tune_c3_check.json
timeout -k 10 300 tools/pmc_kernel.sh gpurun_out/r03tcc_c2 c2 CheckIPHeader base 3,4
