set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/bench_greedy.py --variants 24,27,29,1 --reps 10 > gpurun_out/ptw_exp.log 2>&1
