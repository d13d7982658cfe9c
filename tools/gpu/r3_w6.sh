set -o pipefail
mkdir -p gpurun_out/w6
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rows.py tests/test_gpu_multi.py -k "not beyond" > gpurun_out/w6/tests.log 2>&1 || exit 1
timeout -k 10 300 python tools/rows_ab.py --rows 3700000000 --batch 8000000 --steps 20 --configs "rows@+w4+occ4+occ2" > gpurun_out/w6/c4.log 2>&1 || exit 1
timeout -k 10 300 python tools/rows_ab.py --rows 100000000 --batch 1000000 --steps 50 --configs "rows@+w4" > gpurun_out/w6/c2.log 2>&1 || exit 1
