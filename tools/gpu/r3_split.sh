set -o pipefail
mkdir -p gpurun_out/split
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MBRWT_ROWS_SPLIT=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rows.py -k "not beyond" > gpurun_out/split/tests_split2.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rows.py tests/test_gpu_multi.py -k "not beyond" > gpurun_out/split/tests.log 2>&1 || exit 1
timeout -k 10 300 python tools/rows_ab.py --rows 3700000000 --batch 8000000 --steps 20 --configs "rows@+nosplit+async+async.nosplit" > gpurun_out/split/c4.log 2>&1 || exit 1
timeout -k 10 300 python tools/rows_ab.py --rows 100000000 --batch 2000000 --steps 50 --configs "rows@+nosplit" > gpurun_out/split/c2.log 2>&1 || exit 1
