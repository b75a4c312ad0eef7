#!/bin/bash
# Config 1's element chain with the host glue under a PC sampler (tools only).
#   tools/chain_prof/run.sh build     on the CPU: the glue's host files into
#                                     bin/chain_prof (DWARF 4 line tables)
#   tools/chain_prof/run.sh run       on the GPU box: run it (SAMPLES=file: PC samples);
#                                     resolve.py here
#                                     turns the samples into lines and functions
set -e
D=$(cd "$(dirname "$0")" && pwd); R=$D/../..
B=$D/bin
if [ "$1" = build ]; then
    mkdir -p $B
    F="-O3 -std=c++17 -I$R/include"
    /opt/rocm/bin/hipcc --offload-arch=gfx950 $F -c $R/click_amd/csrc/cksum_api.hip -o $B/api.o
    for f in elements chain ingest; do /opt/rocm/bin/hipcc $F -gdwarf-4 -c $R/click_amd/host/$f.cc -o $B/$f.o; done
    /opt/rocm/bin/hipcc $F -gdwarf-4 -c $D/chain_prof.cc -o $B/main.o
    /opt/rocm/bin/hipcc --offload-arch=gfx950 $B/api.o $B/elements.o $B/chain.o $B/ingest.o $B/main.o -o $B/chain_prof
    rm -f $B/*.o
    python3 -c "import sys; sys.path.insert(0, '$R'); import bench; print(bench.c1_frame().hex())" > $B/frame.hex
else
    cd $B
    ./chain_prof $(cat frame.hex) ${RUNS:-5} ${BATCH:-65536} ${CHAIN:-elements} ${MODE:-staged} ${SEP:-chain}
fi
