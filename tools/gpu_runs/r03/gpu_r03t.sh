#!/bin/bash
# r03t: the driver's bench command itself under rocprofv3 --kernel-trace --stats
O=gpurun_out/r03t; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
