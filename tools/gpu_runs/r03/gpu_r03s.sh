#!/bin/bash
# r03s: IPFragmenter write kernel at 5 / 6 waves per SIMD (fewer loads per lane)
O=gpurun_out/r03s; mkdir -p $O
TUNE_ELEMENT=IPFragmenter timeout -k 10 400 python tools/tune.py --workload c3 --variants base,fwpe5,fu3w5,fu2w6 --rounds 6 > $O/tune_frag.json 2> $O/tune_frag.err
