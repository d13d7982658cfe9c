set -o pipefail
mkdir -p gpurun_out/w2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_wire.py tests/test_gpu_rows.py tests/test_cpp_mirror.py > gpurun_out/w2/tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/bench_wire.py > gpurun_out/w2/bench_wire.log 2>&1 || exit 1
timeout -k 10 200 python tools/rows_ab.py --rows 3700000000 --batch 8000000 --steps 20 --configs "rows@async" > gpurun_out/w2/c4.log 2>&1 || exit 1
