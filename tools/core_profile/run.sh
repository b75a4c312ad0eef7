#!/bin/bash
# The adapter core's own per-packet cost on the CPU (no GPU): the
# measurement program over the null glue, optionally with gprof (-pg).
set -e
D=$(cd "$(dirname "$0")" && pwd); R=$D/../..
mkdir -p $D/bin
g++ -std=c++17 -O2 -g ${PG:+-pg} -I$R/include $R/tests/native/pull_bench.cc $D/null_glue.cc -o $D/bin/pull_bench_null
cd $D/bin && ./pull_bench_null ${1:-1}
if [ -n "$PG" ]; then gprof -b -p ./pull_bench_null gmon.out | head -40; fi
