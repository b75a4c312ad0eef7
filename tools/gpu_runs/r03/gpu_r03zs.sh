#!/bin/bash
# r03zs: the fused packet-stream Set through the dense path on XCD-contiguous
# runs (new default, 4 chunks per lane): every -m gpu test, smoke, the default bench, the C4 profile
O=gpurun_out/r03zs; mkdir -p $O
. tools/gpu_step.sh
step tests timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step bench timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
step prof_c4 timeout -k 10 900 tools/profile.sh r03 c4
