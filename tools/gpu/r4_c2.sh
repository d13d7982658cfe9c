# r04 step C (continued): the two fixed tests, the bench, C3 on the
# variable-length records, C4 odometer A/B (path table vs r03)
set -o pipefail
mkdir -p gpurun_out/r4c
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m "gpu and not slow" tests/test_gpu_dist.py "tests/test_gpu_rows.py::test_auto_layout" "tests/test_gpu_rows.py::test_odometer_walk" > gpurun_out/r4c/tests_fix.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r4c/bench.log 2>&1 || exit 1
timeout -k 10 360 python -u tools/rows_ab.py --rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --steps 10 --configs "rows@async" > gpurun_out/r4c/c3_var.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/rows_ab.py --rows 3700000000 --batch 8000000 --steps 20 --configs "rows@async+w7.async" > gpurun_out/r4c/c4_path_ab.log 2>&1 || exit 1
