# r04 round close, part D (final sources, bench defaults 50 + 10 steps): the -m gpu suite without the slow cases, smoke,
# bench.py (C4, CPU baseline), its kernel trace, the traffic counters (one
# rocprofv3 --pmc pass each), the wire micro-benchmark
set -o pipefail
mkdir -p gpurun_out/r4fd
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m "gpu and not slow" tests > gpurun_out/r4fd/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4fd/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r4fd/bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4fd/prof -o run --output-format csv -- python bench.py --no-cpu --traffic off > gpurun_out/r4fd/bench_prof.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE TCC_EA0_RDREQ_sum; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "k_traverse_rows|k_compact_tiles" -d gpurun_out/r4fd/pmc_$c -o run --output-format csv -- python bench.py --no-cpu --traffic off --steps 5 > gpurun_out/r4fd/pmc_$c.log 2>&1 || exit 1
done
timeout -k 10 200 python -u tools/bench_wire.py > gpurun_out/r4fd/bench_wire.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --workload c3 --no-cpu > gpurun_out/r4fd/bench_c3_q2.log 2>&1 || exit 1
