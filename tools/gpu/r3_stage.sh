set -o pipefail
mkdir -p gpurun_out/stage
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MBRWT_ROWS_STAGE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rows.py -k "not beyond" > gpurun_out/stage/tests.log 2>&1 || exit 1
timeout -k 10 300 python tools/rows_ab.py --rows 3700000000 --batch 8000000 --steps 20 --configs "rows@+stage+stage.occ3+stage.occ4" > gpurun_out/stage/c4.log 2>&1 || exit 1
timeout -k 10 300 python tools/rows_ab.py --rows 100000000 --batch 1000000 --steps 50 --configs "rows@+stage+stage.occ3" > gpurun_out/stage/c2.log 2>&1 || exit 1
