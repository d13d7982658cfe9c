set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MBRWT_ROWS_KERNEL=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rows.py -k "not beyond" > gpurun_out/v4_tests.log 2>&1 || exit 1
timeout -k 10 300 python tools/rows_ab.py --rows 3700000000 --batch 8000000 --steps 20 --configs "rows@+occ3+v4+v4.occ2+v4.occ3" > gpurun_out/v4_c4.log 2>&1 || exit 1
timeout -k 10 300 python tools/rows_ab.py --rows 100000000 --batch 1000000 --steps 50 --configs "rows@+occ3+v4+v4.occ2" > gpurun_out/v4_c2.log 2>&1 || exit 1
