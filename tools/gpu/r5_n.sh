# r05 step N: long records from an LDS copy with the slot's pad word (64 /
# 54 VGPRs); row tests; greedy at 3.7 B; C4; C3 after the revert
set -o pipefail
O=gpurun_out/r5n; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0 --reps 20 --skip-small > $O/greedy_3p7B.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/trav_ab.py --tag c4 > $O/c4.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/trav_ab.py --rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --steps 10 --warmup 3 --tag c3 > $O/c3.log 2>&1 || exit 1
