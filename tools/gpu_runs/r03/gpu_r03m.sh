#!/bin/bash
# r03m: C4 Check cost split (diagnostic libraries built out of tree, results wrong by design)
O=gpurun_out/r03m; mkdir -p $O
TUNE_ELEMENT=CheckUDPHeader timeout -k 10 300 python tools/tune.py --workload c4 --variants base,xNOPC,xNOEAT --rounds 8 > $O/tune_c4_check.json 2> $O/tune_c4_check.err
