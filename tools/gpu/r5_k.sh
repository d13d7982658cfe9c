# r05 step K: compact blocks for non-uniform trees by default; row tests; greedy at 3.7 B
set -o pipefail
O=gpurun_out/r5k; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0 --reps 20 --skip-small > $O/greedy_3p7B.log 2>&1 || exit 1
