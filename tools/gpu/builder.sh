# device builder: parity tests (new + full suite), then the build benchmark at the C2 shape
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
MBRWT_BUILD_TIMING=1 timeout -k 10 600 python -u tools/bench_build.py > gpurun_out/bench_build.log 2>&1
