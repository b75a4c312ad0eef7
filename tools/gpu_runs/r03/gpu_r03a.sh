#!/bin/bash
# Round-3 first GPU check: gpu tests, smoke, default bench, SQ counters of
# the C3 and C4 Check kernels.
set -o pipefail
O=gpurun_out/r03a; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 3
tools/pmc_kernel.sh $O/sq_c4 c4 CheckUDPHeader base 1,2 || exit 4
tools/pmc_kernel.sh $O/sq_c3 c3 CheckUDPHeader base 1,2 || exit 5
