# r04 step B: everything of step A plus row-record export and the AUTO
# default (row records wherever they apply): the whole -m gpu suite without
# the slow cases, the bench, then the C4 full-size parity on row records
set -o pipefail
mkdir -p gpurun_out/r4b
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m "gpu and not slow" tests > gpurun_out/r4b/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r4b/bench.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread -m gpu "tests/test_full_size.py::test_c4_kingsford_rows_full_size" > gpurun_out/r4b/c4_full.log 2>&1 || exit 1
