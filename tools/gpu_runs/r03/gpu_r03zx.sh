#!/bin/bash
# r03zx: XCD-contiguous run order (CLK_XCD_BLOCKS) against the default, per workload
O=gpurun_out/r03zx; mkdir -p $O
. tools/gpu_step.sh
step c4c env TUNE_ELEMENT=CheckUDPHeader timeout -k 10 180 python3 -u tools/tune.py --workload c4 --variants base,xcd --rounds 8 > $O/c4_check.json
step c4s env TUNE_ELEMENT=SetUDPChecksum timeout -k 10 180 python3 -u tools/tune.py --workload c4 --variants base,xcd > $O/c4_set.json
step c3c env TUNE_ELEMENT=CheckUDPHeader timeout -k 10 180 python3 -u tools/tune.py --workload c3 --variants base,xcd > $O/c3_check.json
step c3s env TUNE_ELEMENT=SetUDPChecksum timeout -k 10 180 python3 -u tools/tune.py --workload c3 --variants base,xcd > $O/c3_set.json
step c5c env TUNE_ELEMENT=CheckTCPHeader timeout -k 10 240 python3 -u tools/tune.py --workload c5 --variants base,xcd --rounds 3 > $O/c5_check.json
