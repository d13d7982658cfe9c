# r04 step C: row-record export, the AUTO default and the variable-length
# records of dense rows: the -m gpu suite without the slow cases (the new
# row-record tests last), the bench, the C4 full size on row records, and a
# first C3 A/B (variable-length records against the node image)
set -o pipefail
mkdir -p gpurun_out/r4c
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 420 python -u -m pytest -v --maxfail=5 --timeout 300 --timeout-method thread -m "gpu and not slow" tests/test_gpu_rows.py tests/test_gpu_files.py > gpurun_out/r4c/tests_rows.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest -v --maxfail=5 --timeout 300 --timeout-method thread -m "gpu and not slow" tests --deselect tests/test_gpu_rows.py --deselect tests/test_gpu_files.py > gpurun_out/r4c/tests_rest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r4c/bench.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/rows_ab.py --rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --steps 10 --configs "rows" > gpurun_out/r4c/c3_var.log 2>&1 || exit 1
