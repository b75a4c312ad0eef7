# r05s: thread-owned states without the lock: the core tests, the core's
# legs over the real glue and over the null glue, gprof of the core
set -o pipefail
O=gpurun_out/r05s; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 tests/native/bin/hipcore_test > $O/hipcore_test.log 2>&1
rc=$?; echo "hipcore_test rc=$rc" >> $O/steps.txt; [ $rc -le 1 ] || exit 1
timeout -k 10 300 tests/native/bin/pull_bench > $O/pull.json 2> $O/pull.err || exit 3
echo "pull ok" >> $O/steps.txt
timeout -k 10 200 bash tools/core_profile/run.sh null_run > $O/core_null.json 2>&1 || exit 4
LEG=chain_source REPS=60 TOP=45 timeout -k 10 200 bash tools/core_profile/run.sh gprof_run > $O/core_gprof.txt 2>&1 || exit 5
echo "gprof ok" >> $O/steps.txt
