set -o pipefail
mkdir -p gpurun_out/uni
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py > gpurun_out/uni/tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/rows_ab.py --rows 1000000 --batch 1000000 --steps 50 --configs "rows@+w6+async" > gpurun_out/uni/c2.log 2>&1 || exit 1
timeout -k 10 300 python tools/rows_ab.py --rows 3700000000 --batch 8000000 --steps 20 --configs "rows@+w6+async+w6.async" > gpurun_out/uni/c4.log 2>&1 || exit 1
