# r04 step V: the wire kernels' test over 2..8 segments, 12 / 13 / 32-bit
# fields, and the offsets scan API
set -o pipefail
mkdir -p gpurun_out/r4v
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_wire.py > gpurun_out/r4v/tests_wire.log 2>&1 || exit 1
