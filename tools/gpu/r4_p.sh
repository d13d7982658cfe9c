# r04 step P: the register-based 12-bit label unpack (16-byte loads and stores,
# four tiles per workgroup) and the offsets scan from the packed counts: wire + 2-rank
# tests, the wire micro-benchmark
set -o pipefail
mkdir -p gpurun_out/r4p
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_wire.py tests/test_gpu_dist.py > gpurun_out/r4p/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_wire.py > gpurun_out/r4p/bench_wire.log 2>&1 || exit 1
