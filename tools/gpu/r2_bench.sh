# round 2: the default bench (live PMC traffic, CPU legs incl. RRR-like) and a rocprofv3 kernel summary
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u bench.py --traffic-out gpurun_out/traffic_c4.json > gpurun_out/bench.log 2>&1 || exit 1
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --no-cpu --traffic off --no-probe > "$GRAFT_REPO_ROOT/gpurun_out/bench_rocprof.log" 2>&1
