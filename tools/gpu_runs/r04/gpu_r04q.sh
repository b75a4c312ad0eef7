# r04q: config 1 with the median of five timed runs per leg, then the
# default bench line (its summary carries the C1 medians)
set -o pipefail
O=gpurun_out/r04q; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -c "
import json, click_amd, bench, torch
ctx = click_amd.Context(0)
bench.load_torch_kernels(torch)
print(json.dumps(bench.config1(ctx)))
print(json.dumps(bench.config1_cpu()))
" > $O/c1.json 2> $O/c1.err || exit 4
echo "c1 ok" >> $O/steps.txt
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 5
echo "bench ok" >> $O/steps.txt
