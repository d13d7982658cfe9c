# round 2 (final B): rocprofv3 kernel summaries of the default bench and of the greedy + relax shape (k_traverse_ptw)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --no-cpu --traffic off --no-probe > "$GRAFT_REPO_ROOT/gpurun_out/bench_rocprof.log" 2>&1 &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_greedy" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/bench_greedy.py" --variants 0 --reps 10 --skip-small --scaled-rows 3700000000 --scaled-batch 8000000 > "$GRAFT_REPO_ROOT/gpurun_out/bench_greedy_rocprof.log" 2>&1
