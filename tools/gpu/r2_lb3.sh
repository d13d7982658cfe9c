set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in 1 2 0; do
  MBRWT_LB_MODE=$m timeout -k 10 300 python -u tools/bench_greedy.py --variants 0 --reps 5 --skip-small \
    --scaled-rows 3700000000 --scaled-batch 8000000 > gpurun_out/lb_mode_$m.log 2>&1 || exit 1
done
