# round 2: look-back output path (rowblock kernels write the CSR in place)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "packt or p2w or pack2 or greedy or capacity or errors or overflow or two_streams or null_cols or device_api" > gpurun_out/pytest_lb.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1 &&
timeout -k 10 600 python -u tools/bench_greedy.py --variants 0,20,25 --reps 10 --skip-small \
  --scaled-rows 3700000000 --scaled-batch 8000000 > gpurun_out/bench_greedy_lb.log 2>&1
