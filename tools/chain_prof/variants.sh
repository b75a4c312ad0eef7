#!/bin/bash
# chain_prof builds that differ in compile-time knobs (tools only):
#   tools/chain_prof/variants.sh NAME "FLAGS" ...   on the CPU: bin/chain_prof_NAME
# (the kernels' object is built once and kept in bin/api.o)
set -e
D=$(cd "$(dirname "$0")" && pwd); R=$D/../..
B=$D/bin; mkdir -p $B
F="-O3 -std=c++17 -I$R/include"
[ -f $B/api.o ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 $F -c $R/click_amd/csrc/cksum_api.hip -o $B/api.o
while [ $# -ge 2 ]; do
    name=$1; flags=$2; shift 2
    T=$(mktemp -d)
    for f in elements chain ingest; do /opt/rocm/bin/hipcc $F $flags -gdwarf-4 -c $R/click_amd/host/$f.cc -o $T/$f.o & done
    /opt/rocm/bin/hipcc $F $flags -gdwarf-4 -c $D/chain_prof.cc -o $T/main.o &
    wait
    /opt/rocm/bin/hipcc --offload-arch=gfx950 $B/api.o $T/elements.o $T/chain.o $T/ingest.o $T/main.o -o $B/chain_prof_$name
    rm -rf $T
done
[ -f $B/frame.hex ] || python3 -c "import sys; sys.path.insert(0, '$R'); import bench; print(bench.c1_frame().hex())" > $B/frame.hex
