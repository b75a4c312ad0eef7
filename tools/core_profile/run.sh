#!/bin/bash
# The adapter core's own per-packet cost (tools only).
#   run.sh [SCALE]      on the CPU (no GPU): the measurement program
#                       (tests/native/pull_bench.cc) over the null glue,
#                       with gprof when PG=1
#   run.sh gprof_build  here: pull_bench over the real glue library, linked
#                       (not compiled) with -pg: gprof's PC sampling of the
#                       core's code, no mcount calls; the library's own time
#                       is not sampled
#   run.sh gprof_run    on the GPU box: its chain leg REPS times (LEG=chain_source:
#                       the frames made from a pool as they are pushed), flat profile
#   run.sh null_build   here: the measurement program over the null glue, to
#                       run on the GPU box's host cores (run.sh null_run)
#   run.sh sampler_build  here: the same with sampler.hh in its main file
#                       (bin/pull_bench_null_s; SAMPLES=file when run, then
#                       tools/chain_prof/resolve.py bin/pull_bench_null_s file)
set -e
D=$(cd "$(dirname "$0")" && pwd); R=$D/../..
mkdir -p $D/bin
case "$1" in
gprof_build)
    g++ -std=c++17 -O2 -g -I$R/include -c $R/tests/native/pull_bench.cc -o $D/bin/pull_bench.o
    g++ -pg $D/bin/pull_bench.o -L$R/click_amd -lclick_amd_cksum \
        -L/opt/rocm/lib -Wl,-rpath-link,/opt/rocm/lib -Wl,-rpath,'$ORIGIN/../../../click_amd' \
        -Wl,-rpath,/opt/rocm/lib -o $D/bin/pull_bench_pg
    rm -f $D/bin/pull_bench.o
    ;;
gprof_run)
    cd $D/bin
    ./pull_bench_pg 1 ${LEG:-chain} ${REPS:-100} | tail -2
    gprof -b -p ./pull_bench_pg gmon.out 2>/dev/null | head -${TOP:-40}
    ;;
null_build)
    g++ -std=c++17 -O2 -g -I$R/include $R/tests/native/pull_bench.cc $D/null_glue.cc -o $D/bin/pull_bench_null
    ;;
sampler_build)
    clang=/opt/rocm/llvm/bin/clang++
    $clang -std=c++17 -O2 -gdwarf-4 -I$R/include -include $D/sampler.hh -c $R/tests/native/pull_bench.cc -o $D/bin/pb.o
    $clang -std=c++17 -O2 -gdwarf-4 -I$R/include -c $D/null_glue.cc -o $D/bin/ng.o
    $clang $D/bin/pb.o $D/bin/ng.o -o $D/bin/pull_bench_null_s -ldl
    rm -f $D/bin/pb.o $D/bin/ng.o
    ;;
null_run)
    cd $D/bin && ./pull_bench_null ${1:-1}
    ;;
*)
    g++ -std=c++17 -O2 -g ${PG:+-pg} -I$R/include $R/tests/native/pull_bench.cc $D/null_glue.cc -o $D/bin/pull_bench_null
    cd $D/bin && ./pull_bench_null ${1:-1}
    if [ -n "$PG" ]; then gprof -b -p ./pull_bench_null gmon.out | head -40; fi
    ;;
esac
