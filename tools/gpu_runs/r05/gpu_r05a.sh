# r05a: round-5 baseline on the GPU -- every -m gpu test after the
# addr-check variants left the kernel source, the adapter-core legs
# (pull_bench), and the default bench line
set -o pipefail
O=gpurun_out/r05a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/steps.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 tests/native/bin/pull_bench > $O/pull.json 2> $O/pull.err || exit 3
echo "pull ok" >> $O/steps.txt
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 5
echo "bench ok" >> $O/steps.txt
