set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rows.py -k "not beyond" > gpurun_out/rows_tests.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_c4 -o run --output-format csv -- python tools/rows_ab.py --rows 3700000000 --batch 8000000 --configs "rows@+v3+w5" > gpurun_out/kt_c4.log 2>&1 || exit 1
