# same-box A/B of the traversal (saved build vs in-tree), then the full GPU suite
set -o pipefail
mkdir -p gpurun_out
true
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
