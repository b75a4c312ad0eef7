#!/bin/bash
# deferred gather A/B: glue bursts (glue_ab) and the adapter core's single pushes (pull_bench c3, LD_LIBRARY_PATH)
set -o pipefail
O=$PWD/gpurun_out/r05bj; mkdir -p $O; rm -f $O/core.txt
timeout -k 10 500 python tools/glue_ab.py 3 tools/variants/d0/libclick_amd_cksum.so tools/variants/d256/libclick_amd_cksum.so > $O/ab.txt 2> $O/ab.err || exit 1
for r in 1 2 3; do for v in d0 d256; do
  echo -n "$v " >> $O/core.txt
  LD_LIBRARY_PATH=$PWD/tools/variants/$v timeout -k 10 120 tests/native/bin/pull_bench 1 c3 | python3 -c "import json,sys; print([ (json.loads(l)['leg'], json.loads(l)['mpps']) for l in sys.stdin])" >> $O/core.txt || exit 2
done; done
