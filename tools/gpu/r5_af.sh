# r05 step AF: BASELINE configs[1] (C2, 1 M x 2,652, 1 M-row batch) on the final sources
set -o pipefail
O=gpurun_out/r5af; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u bench.py --workload c2 --no-e2e > $O/bench_c2.log 2>&1 || exit 1
