# round 2: the whole GPU suite (as the driver runs it)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1
