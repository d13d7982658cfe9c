# r04 round close, part C (final sources): the -m gpu suite without the slow
# cases, smoke, bench.py (C4, CPU baseline, live traffic)
set -o pipefail
mkdir -p gpurun_out/r4fc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m "gpu and not slow" tests > gpurun_out/r4fc/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4fc/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r4fc/bench.log 2>&1 || exit 1
