# r04 step I: the tree odometer (rows_walk_tree: any shape) and the compact
# block policy -- row-record walk tests, then the greedy + relax production
# shape at 3.7 B rows (policy's pick, then one row per 64-byte block as r03,
# each with the tree odometer and the stack walk rows_walk4); the VAR decode
# with lanes balanced by units (tests, C3)
set -o pipefail
mkdir -p gpurun_out/r4i
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py -k "odometer or random_matrices or reference_grids or auto_layout or variable" > gpurun_out/r4i/tests.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/rows_ab.py --rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --steps 10 --configs "rows@async" > gpurun_out/r4i/c3.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0,w4 --reps 20 > gpurun_out/r4i/greedy_3p7B.log 2>&1 || exit 1
MBRWT_ROWS_BS=64,1 timeout -k 10 400 python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0,w4 --reps 20 > gpurun_out/r4i/greedy_3p7B_b64s1.log 2>&1 || exit 1
