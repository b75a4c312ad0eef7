#!/bin/bash
# r03j: verify HEAD after the session restart: every -m gpu test, smoke,
# default bench, then C4 / C3 profiles (trace + FETCH/WRITE) and SQ counters
O=gpurun_out/r03j; mkdir -p $O
. tools/gpu_step.sh
step tests timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step bench timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
step prof_c4 timeout -k 10 900 tools/profile.sh r03 c4
step prof_c3 timeout -k 10 900 tools/profile.sh r03 c3
step sq_c4 timeout -k 10 300 tools/pmc_kernel.sh $O/sq_c4 c4 CheckUDPHeader base 1,2
