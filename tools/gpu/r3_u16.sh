set -o pipefail
mkdir -p gpurun_out/u16
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/u16/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/sweep.py --rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --variants 0,20 --reps 10 > gpurun_out/u16/c3_sweep.log 2>&1 || exit 1
timeout -k 10 200 python tools/rows_ab.py --rows 3700000000 --batch 8000000 --steps 20 --configs "rows@async+occ2.async+occ4.async" > gpurun_out/u16/c4_occ.log 2>&1 || exit 1
