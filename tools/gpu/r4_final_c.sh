# r04 round close, part C (final sources): the device wire (register-based
# 12-bit pack and unpack, offsets from the packed counts: wire + 2-rank tests,
# micro-benchmark and its kernel trace), then the -m gpu suite without the
# slow cases, smoke, bench.py (C4, CPU baseline, live traffic)
set -o pipefail
mkdir -p gpurun_out/r4fc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_wire.py tests/test_gpu_dist.py > gpurun_out/r4fc/tests_wire.log 2>&1 || exit 1
timeout -k 10 150 python -u tools/bench_wire.py > gpurun_out/r4fc/bench_wire.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4fc/prof_wire -o wire --output-format csv -- python3 tools/bench_wire.py > gpurun_out/r4fc/bench_wire_prof.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m "gpu and not slow" tests > gpurun_out/r4fc/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4fc/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r4fc/bench.log 2>&1 || exit 1
