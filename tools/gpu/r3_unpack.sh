set -o pipefail
mkdir -p gpurun_out/up
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_wire.py > gpurun_out/up/tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/bench_wire.py > gpurun_out/up/bench_wire.log 2>&1 || exit 1
