# r04 step G: C3 variable-length decode (branchless refill, word-wise label
# counts), lanes per row A/B (G = 4, 8, 16); the VAR tests
set -o pipefail
mkdir -p gpurun_out/r4g
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py -k "variable" > gpurun_out/r4g/tests_var.log 2>&1 || exit 1
for g in 8 16 4; do
MBRWT_VAR_G=$g timeout -k 10 240 python -u tools/rows_ab.py --rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --steps 10 --configs "rows@async" > gpurun_out/r4g/c3_g$g.log 2>&1 || exit 1
done
# the compaction with its direct tiles walked after the copy loop (84 VGPRs)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4g/prof -o bench -- python3 bench.py --no-cpu --traffic off --steps 20 --warmup 5 > gpurun_out/r4g/bench_prof.log 2>&1 || exit 1
