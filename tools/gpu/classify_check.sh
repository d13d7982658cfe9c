# classify: GPU parity (get_labels / get_top_labels, host + device forms, malformed offsets),
# the C++ mirror on the device, benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "get_labels or top_labels" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_cls.log 2>&1 || exit 1
timeout -k 10 300 tests/cpp/_build/test_annotation device > gpurun_out/cpp_annotation_device.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_classify.py --top 10 > gpurun_out/bench_classify_top10.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_classify.py --top 4294967295 --steps 3 > gpurun_out/bench_classify_topall.log 2>&1
