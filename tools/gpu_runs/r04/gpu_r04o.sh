# r04o: host-resident end-to-end rates (bench.py --e2e) for C3 and C2, with
# the adapter-core push and pull legs
set -o pipefail
O=gpurun_out/r04o; mkdir -p $O
timeout -k 10 600 python -u bench.py --e2e --workload c3 > $O/e2e_c3.json 2> $O/e2e_c3.err || exit 2
timeout -k 10 600 python -u bench.py --e2e --workload c2 > $O/e2e_c2.json 2> $O/e2e_c2.err || exit 3
