#!/bin/bash
# r03zr: same-box A/B of the C4 Set: new default (dense path, 4 chunks per
# lane, XCD-contiguous runs) / the same without the XCD order / the old Set
# path with the XCD order / the last commit
O=gpurun_out/r03zr; mkdir -p $O
. tools/gpu_step.sh
step c4s env TUNE_ELEMENT=SetUDPChecksum timeout -k 10 240 python3 -u tools/tune.py --workload c4 --variants base,xcdset0,oldset,prev --rounds 8 > $O/c4_set.json
step c4c env TUNE_ELEMENT=CheckUDPHeader timeout -k 10 180 python3 -u tools/tune.py --workload c4 --variants base,prev --rounds 6 > $O/c4_check.json
