set -o pipefail
mkdir -p gpurun_out/v5
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MBRWT_ROWS_KERNEL=5 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rows.py -k "not beyond" > gpurun_out/v5/tests.log 2>&1 || exit 1
timeout -k 10 300 python tools/rows_ab.py --rows 3700000000 --batch 8000000 --steps 20 --configs "rows@+v5+v5.occ3+v5.occ2+v5.diag1" > gpurun_out/v5/c4.log 2>&1 || exit 1
timeout -k 10 300 python tools/rows_ab.py --rows 100000000 --batch 1000000 --steps 50 --configs "rows@+v5" > gpurun_out/v5/c2.log 2>&1 || exit 1
