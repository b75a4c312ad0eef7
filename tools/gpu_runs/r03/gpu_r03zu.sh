#!/bin/bash
# r03zu: bench with its host work moved out of the gaps between the GPU
# preparation and the warm-ups: bench tests, the default bench, and the
# driver's command under rocprofv3 (per-launch durations)
O=gpurun_out/r03zu; mkdir -p $O
. tools/gpu_step.sh
export TMPDIR=/tmp
step tests timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bench_sizes.py > $O/gpu_tests.log 2>&1
step bench timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
step prof timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err
