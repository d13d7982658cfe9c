set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rows.py tests/test_gpu_multi.py tests/test_cpp_mirror.py -k "not beyond" > gpurun_out/async_tests.log 2>&1 || exit 1
timeout -k 10 300 python tools/rows_ab.py --rows 3700000000 --batch 8000000 --steps 20 --configs "rows@+async" > gpurun_out/async_c4.log 2>&1 || exit 1
timeout -k 10 300 python tools/rows_ab.py --rows 100000000 --batch 1000000 --steps 50 --configs "rows@+async" > gpurun_out/async_c2.log 2>&1 || exit 1
