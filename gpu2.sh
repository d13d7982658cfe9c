set -o pipefail
mkdir -p gpurun_out
(nproc; free -g; lscpu | head -20) > gpurun_out/host.txt 2>&1
timeout -k 10 900 python bench.py > gpurun_out/bench_full.log 2>&1; echo "rc=$?" >> gpurun_out/bench_full.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python bench.py --no-cpu --steps 10 > gpurun_out/prof_trace.log 2>&1; echo "rc=$?" >> gpurun_out/prof_trace.log
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_traverse -d gpurun_out/prof_pmc -o run --output-format csv -- python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/prof_pmc.log 2>&1; echo "rc=$?" >> gpurun_out/prof_pmc.log
