# r05 step X: round close on the final sources -- bench.py (C4, N = 1: live
# PMC traffic, ceilings, CPU baseline, end-to-end leg, whole-batch parity),
# its kernel trace under rocprofv3 --kernel-trace --stats, and the C3 line
set -o pipefail
O=gpurun_out/r5x; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u bench.py --traffic-out $O/traffic_c4.json > $O/bench_c4.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run --output-format csv -- python -u bench.py --no-cpu --no-e2e --no-probe --traffic off > $O/bench_c4_under_rocprof.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --workload c3 --traffic-out $O/traffic_c3.json --no-e2e > $O/bench_c3.log 2>&1 || exit 1
