# r04m: zero-copy vs staged and the output-path / chain tests after the
# IPOutputCombo short-header fix
set -o pipefail
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_zerocopy.py tests/test_gpu_chain.py tests/test_gpu_output_elements.py tests/test_gpu_glue_faults.py tests/test_gpu_adapter_core.py > $O/tests.log 2>&1
