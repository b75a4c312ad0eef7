# r05bv: final check of the tree (chain results queue) -- every -m gpu test, smoke, the core / pull legs,
# the threaded glue, the default bench, the driver's bench command under
# rocprofv3 --kernel-trace --stats, and bench.py --e2e (the C3 push legs
# through the core beside the one-thread CPU leg)
set -o pipefail
O=gpurun_out/r05bv; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/steps.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
echo "smoke ok" >> $O/steps.txt
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 5
echo "bench ok" >> $O/steps.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 10 > $O/bench_prof.json 2> $O/bench_prof.err || exit 6
echo "prof ok" >> $O/steps.txt
timeout -k 10 900 python bench.py --e2e > $O/e2e_c3.json 2> $O/e2e_c3.err || exit 7
echo "e2e ok" >> $O/steps.txt
