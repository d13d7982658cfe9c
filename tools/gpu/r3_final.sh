set -o pipefail
mkdir -p gpurun_out/final
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 100 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || exit 1
timeout -k 10 330 python -u bench.py --traffic-out gpurun_out/final/traffic.json > gpurun_out/final/bench.log 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof -o run --output-format csv -- python bench.py --no-cpu --traffic off --no-probe > gpurun_out/final/bench_under_rocprof.log 2>&1 || exit 1
