#!/bin/bash
# r03b: every GPU test (adapter core, glue retries, dense stream runs, the
# devirtualized glue loops), the glue's per-packet cost, then C4
# stream-kernel variants (dense span path) and the C3 fused Set
O=gpurun_out/r03b; mkdir -p $O
. tools/gpu_step.sh
step tests timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests -o log_cli=false > $O/gpu_tests.log 2>&1
step glue timeout -k 10 120 tools/probes/glue_probe > $O/glue_probe.json 2> $O/glue_probe.err
V=base,span0,spkv1,spkv3,spkv4,spw8,spkv1w8,spw5
step c4check env TUNE_ELEMENT=CheckUDPHeader timeout -k 10 300 python tools/tune.py --workload c4 --variants $V --rounds 6 > $O/tune_c4_check.json 2> $O/tune_c4_check.err
step c4set env TUNE_ELEMENT=SetUDPChecksum timeout -k 10 300 python tools/tune.py --workload c4 --variants base,span0,spkv1,spkv3 --rounds 6 > $O/tune_c4_set.json 2> $O/tune_c4_set.err
step c3set env TUNE_ELEMENT=SetUDPChecksum timeout -k 10 300 python tools/tune.py --workload c3 --variants base,fused,fusednt,fusedsw5 --rounds 6 > $O/tune_c3_set.json 2> $O/tune_c3_set.err
step c1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --workload c2 --no-cpu --no-peak --skip c4,c5 --no-verify > $O/bench_c1.json 2> $O/bench_c1.err
