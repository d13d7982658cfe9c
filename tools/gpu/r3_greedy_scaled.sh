set -o pipefail
mkdir -p gpurun_out/r3g
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u tools/bench_greedy.py --layout rows --variants 0 --skip-small --shapes "greedy+relax" --scaled-rows 3700000000 > gpurun_out/r3g/greedy_rows_scaled.log 2>&1 || exit 1
