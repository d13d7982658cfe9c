# round 2: production tree shape (greedy + relax): shaped-synthetic parity, then
# C2-size and 3.7 B-row measurements of the greedy + relax shape beside the basic one
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "greedy or shaped" > gpurun_out/pytest_shaped.log 2>&1 &&
timeout -k 10 700 python -u tools/bench_greedy.py --variants 0,1,6,10,21 --reps 5 \
  --scaled-rows 3700000000 --scaled-batch 8000000 > gpurun_out/bench_greedy.log 2>&1
