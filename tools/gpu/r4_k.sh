# r04 step K: leaf-parent column lists in the walk table and records longer
# than a block walked per row (not per tile) -- the row-record tests, the
# greedy + relax shape at 3.7 B rows (64-byte blocks of 1 and of 2 rows),
# the C4 bench
set -o pipefail
mkdir -p gpurun_out/r4k
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m "gpu and not slow" tests/test_gpu_rows.py tests/test_gpu_files.py > gpurun_out/r4k/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0,w4 --reps 20 > gpurun_out/r4k/greedy_b64s1.log 2>&1 || exit 1
MBRWT_ROWS_BS=64,2 timeout -k 10 400 python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0 --reps 20 > gpurun_out/r4k/greedy_b64s2.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu > gpurun_out/r4k/bench_c4.log 2>&1 || exit 1
