set -o pipefail
mkdir -p gpurun_out/v3o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MBRWT_ROWS_KERNEL=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py > gpurun_out/v3o/tests_v3.log 2>&1 || exit 1
timeout -k 10 250 python tools/rows_ab.py --rows 3700000000 --batch 8000000 --steps 20 --configs "rows@async+v3.async+async+v3.async" > gpurun_out/v3o/c4.log 2>&1 || exit 1
timeout -k 10 100 python tools/rows_ab.py --rows 1000000 --batch 1000000 --steps 50 --configs "rows@async+v3.async" > gpurun_out/v3o/c2.log 2>&1 || exit 1
