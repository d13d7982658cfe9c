# compaction fast path: GPU parity, then the bench under rocprofv3 kernel stats (raw trace kept in /tmp)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --no-cpu > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run --output-format csv -- python bench.py --no-cpu > gpurun_out/bench_prof.log 2>&1 || exit 1
cp $(find /tmp/prof -name "*kernel_stats.csv" | head -1) gpurun_out/kernel_stats.csv
