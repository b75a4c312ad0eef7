#!/bin/bash
# threaded glue after aligning elements: ZEROCOPY / staged at 1, 2, 4 threads, three rounds
set -o pipefail
O=$PWD/gpurun_out/r05ag; mkdir -p $O; rm -f $O/mt.json
for r in 1 2 3; do
  for m in zerocopy staged; do
    for t in 1 2 4; do
      timeout -k 10 120 tests/native/bin/mt_glue 4194304 CheckIPHeader $m $t >> $O/mt.json 2>> $O/mt.err || exit 1
    done
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_chain.py tests/test_gpu_elements.py tests/test_gpu_threads.py tests/test_gpu_adapter_core.py > $O/tests.log 2>&1 || exit 2
