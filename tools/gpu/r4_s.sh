# r04 step S: the device wire: three-pass offsets scan, register-based 12-bit
# pack and unpack: wire + 2-rank tests, the wire micro-benchmark and its kernel trace
set -o pipefail
mkdir -p gpurun_out/r4s
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_wire.py tests/test_gpu_dist.py > gpurun_out/r4s/tests_wire.log 2>&1 || exit 1
timeout -k 10 150 python -u tools/bench_wire.py > gpurun_out/r4s/bench_wire.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4s/prof -o wire --output-format csv -- python3 tools/bench_wire.py > gpurun_out/r4s/bench_wire_prof.log 2>&1 || exit 1
