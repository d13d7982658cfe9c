set -o pipefail
mkdir -p gpurun_out
make -s -C tests/cpp > gpurun_out/cpp_build.log 2>&1
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log | grep -q "pytest rc=0" || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 900 python bench.py > gpurun_out/bench_full.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python bench.py --no-cpu --steps 10 > gpurun_out/prof_trace.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_traverse_fast2 -d gpurun_out/prof_fetch -o run --output-format csv -- python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/prof_fetch.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_traverse_fast2 -d gpurun_out/prof_write -o run --output-format csv -- python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/prof_write.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum --kernel-include-regex k_traverse_fast2 -d gpurun_out/prof_rdreq -o run --output-format csv -- python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/prof_rdreq.log 2>&1 || exit 1
