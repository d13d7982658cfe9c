# r04 step J: the whole -m gpu suite without the slow cases (tree odometer
# default on non-uniform trees, balanced VAR lanes, 128-byte block cost),
# the greedy + relax shape with 64-byte blocks of 2 rows (159 GB), bench.py
# at C3 (variable-length records, live PMC, whole-batch parity)
set -o pipefail
mkdir -p gpurun_out/r4j
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -q --maxfail=5 --timeout 300 --timeout-method thread -m "gpu and not slow" tests > gpurun_out/r4j/tests.log 2>&1 || exit 1
MBRWT_ROWS_BS=64,2 timeout -k 10 400 python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0 --reps 20 > gpurun_out/r4j/greedy_3p7B_b64s2.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --workload c3 > gpurun_out/r4j/bench_c3.log 2>&1 || exit 1
