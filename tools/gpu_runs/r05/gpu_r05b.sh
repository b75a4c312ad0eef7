# r05b: the chunked core (results delivered in runs of one member): the
# native core test, the adapter-core test, and the core's legs (C3 push
# staged / ZEROCOPY, config 1, pull)
set -o pipefail
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 300 tests/native/bin/hipcore_test > $O/hipcore_test.log 2>&1
rc=$?; echo "hipcore_test rc=$rc" >> $O/steps.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 tests/native/bin/pull_bench > $O/pull.json 2> $O/pull.err || exit 3
echo "pull ok" >> $O/steps.txt
timeout -k 10 300 tests/native/bin/pull_bench 1 c3 >> $O/pull.json 2>> $O/pull.err || exit 4
echo "c3 again ok" >> $O/steps.txt
