#!/bin/bash
# HIP API trace of the threaded glue: ZEROCOPY 1 vs 2 threads, staged 2 threads
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=$PWD/gpurun_out/r05af; mkdir -p $O
for c in "zerocopy 1" "zerocopy 2" "staged 2"; do
  set -- $c
  timeout -k 10 180 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $O/$1_$2 -o run -- tests/native/bin/mt_glue 4194304 CheckIPHeader $1 $2 > $O/$1_$2.json 2> $O/$1_$2.err || exit 1
done
