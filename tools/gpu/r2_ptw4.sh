set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_files.py -x -q --timeout 200 --timeout-method thread \
  -k "packt or greedy" > gpurun_out/pytest_packt.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_greedy.py --variants 0,30,0,30 --reps 10 --skip-small --shapes greedy+relax \
  --scaled-rows 3700000000 --scaled-batch 8000000 > gpurun_out/ptw4.log 2>&1
