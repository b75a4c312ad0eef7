#!/bin/bash
# r03u: packet-stream Check with 5 chunks per lane at 5 waves / 6 at 4
O=gpurun_out/r03u; mkdir -p $O
TUNE_ELEMENT=CheckUDPHeader timeout -k 10 300 python tools/tune.py --workload c4 --variants base,dk5,dk6w4 --rounds 8 > $O/tune_c4_check.json 2> $O/tune_c4_check.err
