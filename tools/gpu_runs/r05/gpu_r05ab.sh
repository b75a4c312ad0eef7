#!/bin/bash
# full GPU tests + bench after the chain push / loop changes
set -o pipefail
O=$PWD/gpurun_out/r05ab; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 2
timeout -k 10 900 python bench.py --e2e > $O/e2e.json 2> $O/e2e.err || exit 3
