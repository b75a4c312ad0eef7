#!/bin/bash
# Profile bench.py on the GPU box (run through gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats         (per-kernel durations)
#   2. rocprofv3 --pmc FETCH_SIZE   (own pass)  (HBM read bytes)
#   3. rocprofv3 --pmc WRITE_SIZE   (own pass)  (HBM write bytes)
# then tools/pmc_summary.py writes profiles/<tag>/ and profiles/pmc_<wl>.json.
# Usage: tools/profile.sh <tag> <workload> [bench args...]
set -euo pipefail
TAG=$1; WL=$2; shift 2
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG}_${WL}
mkdir -p "$OUT"
# FRAG=1 keeps the IPFragmenter section (C3 only)
NOFRAG=--no-frag; [ "${FRAG:-0}" = 1 ] && NOFRAG=
ARGS="--workload $WL --no-cpu --no-peak --no-c2 --no-c1 $NOFRAG --skip c4,c5 $*"
# summaries land in gpurun_out/profiles/ (merged back); copy them into profiles/
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --steps 20 --warmup 10 $ARGS > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 bench.py --steps 3 --warmup 1 $ARGS > "$OUT/bench_fetch.json" 2> "$OUT/bench_fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 bench.py --steps 3 --warmup 1 $ARGS > "$OUT/bench_write.json" 2> "$OUT/bench_write.err"
# 4. the write requests by class (whole 64 B vs partial), own pass
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d "$OUT/wrreq" -o run -- \
    python3 bench.py --steps 3 --warmup 1 $ARGS > "$OUT/bench_wrreq.json" 2> "$OUT/bench_wrreq.err"
python3 tools/pmc_summary.py "$OUT" "$TAG" "$WL" gpurun_out/profiles 20
