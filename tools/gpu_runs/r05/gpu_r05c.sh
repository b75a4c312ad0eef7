# r05c: the core's legs with config 1 pushed from a packet pool as it is
# made (InfiniteSource-like) beside the pre-made frames
set -o pipefail
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 300 tests/native/bin/pull_bench > $O/pull.json 2> $O/pull.err || exit 3
echo "pull ok" >> $O/steps.txt
