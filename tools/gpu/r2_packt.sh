# round 2: KIND_PACKT images + k_traverse_ptw -- new tests first, then the
# parity / files suites, then the greedy shape at C2 and 3.7 B rows
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "packt" > gpurun_out/pytest_packt.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_files.py -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_parity_files.log 2>&1 &&
timeout -k 10 500 python -u tools/bench_greedy.py --variants 0,1,24,25,26,28 --reps 5 \
  --scaled-rows 3700000000 --scaled-batch 8000000 > gpurun_out/bench_greedy_packt.log 2>&1
