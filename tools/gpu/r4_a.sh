# r04 step A: rows cleanup (direct pass folded into the compaction), wire pack
# capacity, new parity tests (C2 over both layouts, classify on rows vs the
# reference semantics, C4 full size on rows), then the bench
set -o pipefail
mkdir -p gpurun_out/r4a
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rows.py tests/test_gpu_wire.py tests/test_capi.py "tests/test_gpu_parity.py::test_c2_kingsford_small_exact" > gpurun_out/r4a/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r4a/bench.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread -m gpu "tests/test_full_size.py::test_c4_kingsford_rows_full_size" > gpurun_out/r4a/c4_full.log 2>&1 || exit 1
