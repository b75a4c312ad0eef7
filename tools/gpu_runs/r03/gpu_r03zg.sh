#!/bin/bash
# r03zg: closing check after the XCD-ordered Set: every -m gpu test, smoke, default bench
O=gpurun_out/r03zg; mkdir -p $O
. tools/gpu_step.sh
step tests timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step bench timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
