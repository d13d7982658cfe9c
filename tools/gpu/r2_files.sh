# round 2: device image export / BRWT stream load on the GPU, C++ mirror (load/serialize) on the device
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_files.py tests/test_cpp_mirror.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_files.log 2>&1
