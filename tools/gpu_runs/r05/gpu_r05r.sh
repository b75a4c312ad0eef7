# r05r: every -m gpu test (the converging-outputs scenario, chains
# double-buffered), the adapter core's own cost over the null glue on this
# box's host, and gprof of the core over the real glue (chain leg, pooled
# source)
set -o pipefail
O=gpurun_out/r05r; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/steps.txt; [ $rc -le 1 ] || exit 1
timeout -k 10 120 tests/native/bin/hipcore_test > $O/hipcore_test.log 2>&1 || exit 2
timeout -k 10 200 bash tools/core_profile/run.sh null_run > $O/core_null.json 2>&1 || exit 3
echo "null ok" >> $O/steps.txt
LEG=chain_source REPS=60 TOP=45 timeout -k 10 200 bash tools/core_profile/run.sh gprof_run > $O/core_gprof.txt 2>&1 || exit 4
echo "gprof ok" >> $O/steps.txt
