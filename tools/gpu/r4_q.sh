# r04 step Q: step P (wire tests, wire micro-benchmark), then the slow
# -m gpu cases (C3 / C4 / C5 at full size, rows >= 2^32)
set -o pipefail
mkdir -p gpurun_out/r4q
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_wire.py tests/test_gpu_dist.py > gpurun_out/r4q/tests_wire.log 2>&1 || exit 1
timeout -k 10 150 python -u tools/bench_wire.py > gpurun_out/r4q/bench_wire.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread -m "gpu and slow" tests > gpurun_out/r4q/pytest_gpu_slow.log 2>&1 || exit 1
