# r04 round close, part B: the slow -m gpu cases (C3 / C4 / C5 at full size,
# rows >= 2^32)
set -o pipefail
mkdir -p gpurun_out/r4fb
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1100 python -u -m pytest -v --timeout 600 --timeout-method thread -m "gpu and slow" tests > gpurun_out/r4fb/pytest_gpu_slow.log 2>&1 || exit 1
