# r04 step W: the compact row-record footprint build option (test, and the
# greedy + relax shape at 3.7 B rows built compact)
set -o pipefail
mkdir -p gpurun_out/r4w
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py -k "compact or tree_odometer or auto_layout" > gpurun_out/r4w/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0 --reps 20 --compact > gpurun_out/r4w/greedy_compact.log 2>&1 || exit 1
