set -o pipefail
mkdir -p gpurun_out/r3g gpurun_out/sc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u tools/bench_greedy.py --layout rows --variants 0 --scaled-rows 3700000000 > gpurun_out/r3g/greedy_rows.log 2>&1 || exit 1
timeout -k 10 400 python tools/rows_ab.py --rows 4500000000 --batch 8000000 --steps 20 --configs "rows@+async" > gpurun_out/sc/rows_4p5B.log 2>&1 || exit 1
