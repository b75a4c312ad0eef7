# r05q: why the split fragmenter (headers pass, then payloads) is slower:
# HBM write requests, whole 64 B vs partial, base against fsplit
set -o pipefail
O=gpurun_out/r05q; mkdir -p $O
export TMPDIR=/tmp TUNE_ELEMENT=IPFragmenter
for v in base fsplit; do
  for set in "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "FETCH_SIZE"; do
    tag=$(echo $set | cut -d' ' -f1)
    timeout -s KILL 300 rocprofv3 --pmc $set --output-format csv -d $O/${v}_$tag -o run -- python3 tools/tune.py --workload c3 --variants $v --rounds 1 --launches 2 > $O/${v}_$tag.log 2>&1 || exit 1
  done
done
echo ok >> $O/steps.txt
