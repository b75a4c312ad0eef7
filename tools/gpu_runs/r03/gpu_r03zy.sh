#!/bin/bash
# r03zy: the fused packet-stream Set on XCD-contiguous runs (default) against
# the dealt order; the all-kernels switch on C2's writing elements; then every
# -m gpu test, smoke and the default bench on the new default
O=gpurun_out/r03zy; mkdir -p $O
. tools/gpu_step.sh
step c4s env TUNE_ELEMENT=SetUDPChecksum timeout -k 10 180 python3 -u tools/tune.py --workload c4 --variants base,xcdset0 --rounds 8 > $O/c4_set.json
step c2s env TUNE_ELEMENT=SetIPChecksum timeout -k 10 120 python3 -u tools/tune.py --workload c2 --variants base,xcd > $O/c2_set.json
step c2t env TUNE_ELEMENT=DecIPTTL timeout -k 10 120 python3 -u tools/tune.py --workload c2 --variants base,xcd > $O/c2_ttl.json
step tests timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step bench timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
