#!/bin/bash
# r03o: Check kernels parsing the header from the pass-0 chunk registers
# (no header loads of their own): C3 / C5 time, and C3 L2->HBM read requests
O=gpurun_out/r03o; mkdir -p $O
. tools/gpu_step.sh
step c3 env TUNE_ELEMENT=CheckUDPHeader timeout -k 10 300 python tools/tune.py --workload c3 --variants base,hdrc --rounds 10 > $O/tune_c3_check.json 2> $O/tune_c3_check.err
step c5 env TUNE_ELEMENT=CheckTCPHeader timeout -k 10 300 python tools/tune.py --workload c5 --variants base,hdrc --rounds 4 > $O/tune_c5_check.json 2> $O/tune_c5_check.err
step pmc_base timeout -k 10 300 tools/pmc_kernel.sh $O/pmc_base c3 CheckUDPHeader base 3
step pmc_hdrc timeout -k 10 300 tools/pmc_kernel.sh $O/pmc_hdrc c3 CheckUDPHeader hdrc 3
