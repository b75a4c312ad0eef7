#!/bin/bash
# Build the library from the last commit's sources into build/variants/lib_prev.so
# (the "prev" variant of tools/tune.py: an A/B against the working tree).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
cd "$ROOT"
for f in $(git ls-files click_amd/csrc click_amd/host include); do
    mkdir -p "$T/$(dirname "$f")"
    git show "HEAD:$f" > "$T/$f"
done
mkdir -p build/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I"$T/include" \
    -o build/variants/lib_prev.so "$T/click_amd/csrc/cksum_api.hip" "$T/click_amd/host/elements.cc" "$T/click_amd/host/ingest.cc"
rm -rf "$T"
