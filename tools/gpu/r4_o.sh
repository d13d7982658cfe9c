# r04 step O (+ P): the tree odometer in workgroups of 11 waves where the walk
# table leaves room (22 instead of 16 waves per CU): row tests, the greedy +
# relax shape at 3.7 B rows (one and two rows per 64-byte block)
set -o pipefail
mkdir -p gpurun_out/r4o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m "gpu and not slow" tests/test_gpu_rows.py > gpurun_out/r4o/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0 --reps 20 > gpurun_out/r4o/greedy_b64s1.log 2>&1 || exit 1
MBRWT_ROWS_BS=64,2 timeout -k 10 400 python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0 --reps 20 > gpurun_out/r4o/greedy_b64s2.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_wire.py tests/test_gpu_dist.py > gpurun_out/r4o/tests_wire.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_wire.py > gpurun_out/r4o/bench_wire.log 2>&1 || exit 1
