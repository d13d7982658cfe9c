# Full GPU round: parity suite, smoke, bench (whole-batch parity + CPU baseline),
# kernel-trace stats, and one rocprofv3 --pmc pass per counter (separate runs).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --no-cpu > gpurun_out/bench_prof.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE TCC_EA0_RDREQ_sum; do
  timeout -s KILL 300 rocprofv3 --pmc $c -d gpurun_out/pmc_$c -o run --output-format csv -- python bench.py --no-cpu --steps 5 > gpurun_out/pmc_$c.log 2>&1 || exit 1
done
