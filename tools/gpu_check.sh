# GPU box: the given pytest selection, then optional bench workloads.
# Usage: bash tools/gpu_check.sh "<pytest -k expr or ''>" [workload ...]
set -o pipefail
mkdir -p gpurun_out
K="$1"; shift
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 120 --timeout-method thread \
      > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
for wl in "$@"; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu --no-peak --no-c2 --steps 10 \
      > gpurun_out/bench_$wl.json 2> gpurun_out/bench_$wl.err || { tail -20 gpurun_out/bench_$wl.err; exit 2; }
done
