set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_files.py -x -q --timeout 200 --timeout-method thread \
  -k "packt or greedy" > gpurun_out/pytest_packt.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_greedy.py --variants 0,30 --reps 10 --skip-small --shapes greedy+relax \
  --scaled-rows 3700000000 --scaled-batch 8000000 > gpurun_out/ptw3.log 2>&1 &&
cd /tmp &&
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  --kernel-include-regex k_traverse_ptw -d "$GRAFT_REPO_ROOT/gpurun_out/sq3" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/tools/bench_greedy.py" --variants 0 --reps 2 --skip-small --shapes greedy+relax \
  --scaled-rows 3700000000 --scaled-batch 8000000 > "$GRAFT_REPO_ROOT/gpurun_out/sq3.log" 2>&1
