# round 2: compaction A/B (16 lanes vs one wave per rowblock) and SQ counters of k_traverse_ptw
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/bench_greedy.py --variants 0 --reps 10 --skip-small --scaled-rows 3700000000 \
  --scaled-batch 8000000 > gpurun_out/compact_default.log 2>&1 &&
MBRWT_COMPACT=w timeout -k 10 300 python -u tools/bench_greedy.py --variants 0 --reps 10 --skip-small \
  --scaled-rows 3700000000 --scaled-batch 8000000 > gpurun_out/compact_wave.log 2>&1 &&
cd /tmp &&
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  --kernel-include-regex k_traverse_ptw -d "$GRAFT_REPO_ROOT/gpurun_out/sq1" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/tools/bench_greedy.py" --variants 0 --reps 2 --skip-small --shapes greedy+relax \
  --scaled-rows 3700000000 --scaled-batch 8000000 > "$GRAFT_REPO_ROOT/gpurun_out/sq1.log" 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY \
  --kernel-include-regex k_traverse_ptw -d "$GRAFT_REPO_ROOT/gpurun_out/sq2" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/tools/bench_greedy.py" --variants 0 --reps 2 --skip-small --shapes greedy+relax \
  --scaled-rows 3700000000 --scaled-batch 8000000 > "$GRAFT_REPO_ROOT/gpurun_out/sq2.log" 2>&1
