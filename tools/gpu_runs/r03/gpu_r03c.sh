#!/bin/bash
# r03c: all GPU tests (glue staging change, fused run-block Set), C4
# dense-span variants without pipelining, C3 / C5 fused run-block Set,
# config 1 + C2 E2E glue rates
O=gpurun_out/r03c; mkdir -p $O
. tools/gpu_step.sh
step tests timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
step glue timeout -k 10 120 tools/probes/glue_probe > $O/glue_probe.json 2> $O/glue_probe.err
step c4check env TUNE_ELEMENT=CheckUDPHeader timeout -k 10 300 python tools/tune.py --workload c4 --variants span0,spnp,spnp3,spnp4w5,span0w5 --rounds 6 > $O/tune_c4_check.json 2> $O/tune_c4_check.err
step c3set env TUNE_ELEMENT=SetUDPChecksum timeout -k 10 300 python tools/tune.py --workload c3 --variants base,fused,fusedrb0 --rounds 8 > $O/tune_c3_set.json 2> $O/tune_c3_set.err
step c5set env TUNE_ELEMENT=SetTCPChecksum timeout -k 10 300 python tools/tune.py --workload c5 --variants base,fused --rounds 4 > $O/tune_c5_set.json 2> $O/tune_c5_set.err
step c1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --workload c2 --no-cpu --no-peak --skip c4,c5 --no-verify > $O/bench_c1.json 2> $O/bench_c1.err
step e2e timeout -k 10 400 python bench.py --e2e --workload c2 > $O/e2e_c2.json 2> $O/e2e_c2.err
step pmc_c4 timeout -k 10 400 tools/pmc_kernel.sh $O/pmc_c4 c4 CheckUDPHeader span0 3,4
step pmc_c3 timeout -k 10 400 tools/pmc_kernel.sh $O/pmc_c3 c3 CheckUDPHeader base 3,4
