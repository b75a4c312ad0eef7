#!/bin/bash
# r03zw: the dense path for the fused Set, now on XCD-contiguous runs; the C4
# profile (trace + FETCH_SIZE + WRITE_SIZE passes) for the new Set order
O=gpurun_out/r03zw; mkdir -p $O
. tools/gpu_step.sh
step c4s env TUNE_ELEMENT=SetUDPChecksum timeout -k 10 180 python3 -u tools/tune.py --workload c4 --variants base,dset,dsetk4 > $O/c4_set_dense.json
step prof_c4 timeout -k 10 900 tools/profile.sh r03 c4
