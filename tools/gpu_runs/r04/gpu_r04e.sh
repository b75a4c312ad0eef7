# r04e: every -m gpu test (adapter classes, pull double-buffering, per-thread
# delivery, descriptor past max_len, ZEROCOPY abandon at every step) and smoke
set -o pipefail
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_adapter_core.py > $O/adapter.log 2>&1
echo "adapter rc=$?" >> $O/steps.txt
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
echo "tests rc=$?" >> $O/steps.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
