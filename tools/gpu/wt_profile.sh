# C5 (BinRel-WT) profile: kernel-trace stats and one rocprofv3 --pmc pass per counter
# (raw traces are reduced to the decode kernel's rows: gpurun copies back <= 64 MiB)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/wtprof -o run --output-format csv -- python tools/bench_binrel_wt.py --no-cpu --check-rows 1000 > gpurun_out/wt_prof.log 2>&1 || exit 1
cp /tmp/wtprof/run_kernel_stats.csv gpurun_out/wt_kernel_stats.csv
for c in FETCH_SIZE WRITE_SIZE TCC_EA0_RDREQ_sum; do
  timeout -s KILL 400 rocprofv3 --pmc $c -d /tmp/wtpmc_$c -o run --output-format csv -- python tools/bench_binrel_wt.py --no-cpu --check-rows 1000 --steps 2 > gpurun_out/wtpmc_$c.log 2>&1 || exit 1
  (head -1 /tmp/wtpmc_$c/run_counter_collection.csv; grep "k_wt_decode" /tmp/wtpmc_$c/run_counter_collection.csv) > gpurun_out/wtpmc_$c.csv
done
