# r04 round close, part E (final sources): every -m gpu test (slow cases
# included), smoke, bench.py with its defaults
set -o pipefail
mkdir -p gpurun_out/r4fe
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/r4fe/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4fe/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r4fe/bench.log 2>&1 || exit 1
