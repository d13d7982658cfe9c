# r05 step J: spill cost by walk family (C4 keeps two rows per block; the
# greedy + relax shape takes the compact blocks by default); bench
set -o pipefail
O=gpurun_out/r5j; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/trav_ab.py --tag release > $O/c4_release.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0 --reps 20 --skip-small > $O/greedy_3p7B.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --traffic off > $O/bench.log 2>&1 || exit 1
