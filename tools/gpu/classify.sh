# batched get_labels (classify): parity tests, then the bench at ratio 0 and 0.5
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k get_labels -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_cls.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_classify.py > gpurun_out/bench_classify.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_classify.py --ratio 0.5 --steps 3 > gpurun_out/bench_classify_r05.log 2>&1
