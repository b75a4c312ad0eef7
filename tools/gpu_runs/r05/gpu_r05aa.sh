#!/bin/bash
# bench + e2e after the glue-loop inlining
set -o pipefail
O=$PWD/gpurun_out/r05aa; mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 900 python bench.py --e2e > $O/e2e.json 2> $O/e2e.err || exit 2
