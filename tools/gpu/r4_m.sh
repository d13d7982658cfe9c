# r04 step M: which streams overlap (two pool streams vs the null stream +
# a pool stream), bench.py --query-streams 2 with the whole-batch parity
set -o pipefail
mkdir -p gpurun_out/r4m
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/overlap_ab.py --steps 40 > gpurun_out/r4m/overlap.log 2>&1 || exit 1
timeout -k 10 500 python -u bench.py --traffic off --steps 30 --query-streams 2 > gpurun_out/r4m/bench_q2_parity.log 2>&1 || exit 1
