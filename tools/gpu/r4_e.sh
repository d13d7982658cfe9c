# r04 step E: C3 on the variable-length records (ranged build) with G A/B,
# the C4 odometer A/B (path table vs r03's), a rocprofv3 kernel trace of the
# C4 bench (where the step's time goes)
set -o pipefail
mkdir -p gpurun_out/r4e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 420 python -u tools/rows_ab.py --rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --steps 10 --configs "rows@async" > gpurun_out/r4e/c3_var.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/rows_ab.py --rows 3700000000 --batch 8000000 --steps 20 --configs "rows@async+w7.async" > gpurun_out/r4e/c4_path_ab.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4e/prof -o bench -- python3 bench.py --no-cpu --traffic off --steps 20 --warmup 5 > gpurun_out/r4e/bench_prof.log 2>&1 || exit 1
