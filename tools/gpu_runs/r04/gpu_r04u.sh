# r04u: check of the tree -- every -m gpu test, smoke, the pull legs,
# config 1 (elements, combos, chains), the default bench, and the driver's
# bench command under rocprofv3 --kernel-trace --stats
set -o pipefail
O=gpurun_out/r04u; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/steps.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
echo "smoke ok" >> $O/steps.txt
timeout -k 10 300 tests/native/bin/pull_bench > $O/pull.json 2> $O/pull.err || exit 3
timeout -k 10 600 python -u -c "
import json, click_amd, bench, torch
ctx = click_amd.Context(0)
bench.load_torch_kernels(torch)
print(json.dumps(bench.config1(ctx)))
" > $O/c1.json 2> $O/c1.err || exit 4
echo "c1 ok" >> $O/steps.txt
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 5
echo "bench ok" >> $O/steps.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 10 > $O/bench_prof.json 2> $O/bench_prof.err || exit 6
echo "prof ok" >> $O/steps.txt
