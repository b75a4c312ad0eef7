#!/bin/bash
# r03h: diagnostics of the dense stream path (results of x* variants are wrong by design)
O=gpurun_out/r03h; mkdir -p $O
. tools/gpu_step.sh
step c4check env TUNE_ELEMENT=CheckUDPHeader timeout -k 10 300 python tools/tune.py --workload c4 --variants base,ahead0,xnoeat,xnoeat0,xdefld,dense0 --rounds 5 > $O/tune_c4_check.json 2> $O/tune_c4_check.err
step pmc_base timeout -k 10 300 tools/pmc_kernel.sh $O/pmc_base c4 CheckUDPHeader base 1,2
step pmc_dense0 timeout -k 10 300 tools/pmc_kernel.sh $O/pmc_dense0 c4 CheckUDPHeader dense0 1,2
