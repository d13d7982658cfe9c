set -o pipefail
mkdir -p gpurun_out/final
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u bench.py --traffic-out gpurun_out/final/traffic.json > gpurun_out/final/bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof -o run --output-format csv -- python bench.py --no-cpu --traffic off --no-probe > gpurun_out/final/bench_under_rocprof.log 2>&1 || exit 1
