# classify over both schemes: GPU parity (Python) and the C++ mirror on the device
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_binrel_wt.py tests/test_gpu_parity.py -k "classify or get_labels or top_labels" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_wt_cls.log 2>&1 || exit 1
timeout -k 10 300 tests/cpp/_build/test_annotation device > gpurun_out/cpp_annotation_device.log 2>&1 || exit 1
timeout -k 10 300 tests/cpp/_build/test_binrel_wt device > gpurun_out/cpp_binrel_wt_device.log 2>&1
