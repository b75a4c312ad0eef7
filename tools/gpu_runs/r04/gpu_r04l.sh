# r04l: the multi-rank bench rehearsals (two gloo ranks on one GPU, RCCL
# with one rank) with the root-scatter sample
set -o pipefail
O=gpurun_out/r04l; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_bench_sizes.py -k "ranks or rccl or world" > $O/tests.log 2>&1
