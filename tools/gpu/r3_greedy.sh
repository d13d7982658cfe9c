set -o pipefail
mkdir -p gpurun_out/r3g
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_binrel_wt.py tests/test_cpp_mirror.py tests/test_gpu_shards.py > gpurun_out/r3g/tests.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_greedy.py --layout rows --variants 0 > gpurun_out/r3g/greedy_rows_c2.log 2>&1 || exit 1
