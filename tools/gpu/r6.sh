# r06 GPU steps (run from the repo root:
#   /usr/local/graft/bin/gpurun --timeout 900 -- bash tools/gpu/r6.sh STAGE [STAGE ...])
# Every GPU step has its own time limit, steps chain with &&, a heartbeat
# file shows progress.  Outputs: gpurun_out/r6_STAGE/ (copied to profiles/r06/).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
( for i in $(seq 1 30); do sleep 60; echo "heartbeat $i $(date +%T)" >> gpurun_out/r6_heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
B="python -u bench.py --no-e2e --no-probe --traffic off"
for STAGE in "$@"; do
O=gpurun_out/r6_$STAGE; mkdir -p $O
case "$STAGE" in
rows)  # the row-record GPU tests + host pipeline + classes
  timeout -k 10 700 $PYT tests/test_gpu_rows.py tests/test_gpu_hostpipe.py tests/test_gpu_classes.py > $O/pytest_rows.log 2>&1
  ;;
trace)  # C4 bench (live PMC, ceilings) and the kernel trace of its two-stream timed region
  timeout -k 10 400 python -u bench.py --no-cpu --no-e2e --traffic-out $O/traffic_c4.json > $O/bench_c4.log 2>&1 &&
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run --output-format csv -- python -u bench.py --no-cpu --no-e2e --no-probe --traffic off --steps 50 > $O/bench_c4_under_rocprof.log 2>&1 &&
  python tools/trace_overlap.py $(find $O/prof_c4 -name "*kernel_trace.csv" | head -1) > $O/overlap.json 2>&1
  ;;
greedy)  # the greedy + relax shape at 3.7 B rows: the automatic block shape and the alternatives
  timeout -k 10 900 python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0 --reps 10 --skip-small --blocks auto,128:3,64:1 > $O/greedy_blocks.log 2>&1
  ;;
nib)  # nibble-coded records: the row-record tests, C4 with nibble codes (parity) and bytes (A/B)
  timeout -k 10 700 $PYT tests/test_gpu_rows.py tests/test_gpu_classes.py tests/test_gpu_files.py > $O/pytest_rows.log 2>&1 &&
  timeout -k 10 400 python -u bench.py --no-e2e --traffic off --rows-code 1 > $O/bench_c4_nib.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu --rows-code 0 > $O/bench_c4_byte.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu --rows-code 1 > $O/bench_c4_nib2.log 2>&1
  ;;
nib2)  # nibble decode with one 4-byte LDS read: the nibble tests, C4 nibble (parity) / byte A/B
  timeout -k 10 700 $PYT tests/test_gpu_rows.py -k "nibble or odometer or async or errors" > $O/pytest_rows.log 2>&1 &&
  timeout -k 10 400 python -u bench.py --no-e2e --traffic off --rows-code 1 > $O/bench_c4_nib.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu --rows-code 0 > $O/bench_c4_byte.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu --rows-code 1 > $O/bench_c4_nib2.log 2>&1
  ;;
wide)  # row records for nodes up to 64 wide and up to 2^16 columns; the row-record suite
  timeout -k 10 900 $PYT tests/test_gpu_rows.py tests/test_gpu_classes.py tests/test_gpu_files.py tests/test_gpu_parity.py > $O/pytest_rows.log 2>&1
  ;;
cumask)  # VERDICT r05 #1a: the compaction on a CU-masked stream -- its test, then ABAB C4 steps
  timeout -k 10 300 $PYT tests/test_gpu_rows.py -k "compact_cus or async or errors" > $O/pytest_rows.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu --compact-cus 0 > $O/bench_c4_cus0_1.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu --compact-cus 8 > $O/bench_c4_cus8_1.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu --compact-cus 0 > $O/bench_c4_cus0_2.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu --compact-cus 8 > $O/bench_c4_cus8_2.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu --compact-cus 4 > $O/bench_c4_cus4.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu --compact-cus 16 > $O/bench_c4_cus16.log 2>&1
  ;;
qstreams)  # C4 with 2 / 3 / 4 query streams (contexts sharing the image), ABAB
  timeout -k 10 200 $B --no-cpu --query-streams 2 > $O/bench_c4_q2_1.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu --query-streams 3 > $O/bench_c4_q3_1.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu --query-streams 2 > $O/bench_c4_q2_2.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu --query-streams 3 > $O/bench_c4_q3_2.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu --query-streams 4 > $O/bench_c4_q4.log 2>&1
  ;;
final_tests)  # the round's records, 1/3: every -m gpu test but the full-size ones, smoke
  timeout -k 10 1000 $PYT -q tests -m "gpu and not slow" -x > $O/pytest_gpu_not_slow.log 2>&1 &&
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  ;;
final_slow)  # 2/3: the full-size parity cases (C3, C4, C5, rows >= 2^32)
  timeout -k 10 1100 $PYT tests -m "gpu and slow" -x > $O/pytest_gpu_slow.log 2>&1
  ;;
final_bench)  # 3/3: bench.py (whole-batch parity, CPU baseline, live PMC), its kernel trace + stats
  timeout -k 10 400 python -u bench.py --traffic-out $O/traffic_c4.json > $O/bench_c4.log 2>&1 &&
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run --output-format csv -- python -u bench.py --no-cpu --no-e2e --no-probe --traffic off > $O/bench_c4_under_rocprof.log 2>&1
  ;;
greedy_sq)  # SQ / TA counters of the greedy + relax traversal at 3.7 B rows (three passes, r05's C4 sets)
  G="python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0 --reps 3 --skip-small"
  timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $O/sq1 -o run --output-format csv -- $G > $O/sq1.log 2>&1 &&
  timeout -s KILL 400 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $O/sq2 -o run --output-format csv -- $G > $O/sq2.log 2>&1 &&
  timeout -s KILL 400 rocprofv3 --pmc GRBM_COUNT GRBM_GUI_ACTIVE SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_WR TA_BUFFER_WAVEFRONTS_sum TA_TA_BUSY_sum -d $O/sq3 -o run --output-format csv -- $G > $O/sq3.log 2>&1
  ;;
rehearsal)  # bench.py's N > 1 step on the final sources: two ranks on one GPU over gloo, 1 B rows (two images fit)
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --dist-backend gloo --rows 1000000000 --steps 10 --warmup 3 --no-e2e > $O/rehearsal_2rank.log 2>&1
  ;;
term)  # terminal records: their tests, C4 with them (parity) and ABAB against bytes, the greedy shape with both
  timeout -k 10 500 $PYT tests/test_gpu_rows.py -k "terminal or nibble or odometer or async or errors or compact_cus" > $O/pytest_rows.log 2>&1 &&
  timeout -k 10 300 python -u bench.py --no-e2e --no-probe --traffic off --rows-code 2 > $O/bench_c4_term_parity.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu --rows-code 0 > $O/bench_c4_byte_1.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu --rows-code 2 > $O/bench_c4_term_1.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu --rows-code 0 > $O/bench_c4_byte_2.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu --rows-code 2 > $O/bench_c4_term_2.log 2>&1 &&
  timeout -k 10 600 python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0 --reps 10 --skip-small --rows-codes 0,2 > $O/greedy_codes.log 2>&1
  ;;
greedy_default)  # the greedy + relax shape at 3.7 B rows with the library defaults (AUTO records)
  timeout -k 10 600 python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0 --reps 10 --skip-small > $O/greedy_default.log 2>&1
  ;;
final_rest)  # the files after a first failure in test_gpu_rows.py, smoke, then the full-size cases
  timeout -k 10 900 $PYT -q tests/test_gpu_rows.py tests/test_gpu_shards.py tests/test_gpu_wire.py -m "gpu and not slow" > $O/pytest_rest.log 2>&1 &&
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
  timeout -k 10 900 $PYT tests -m "gpu and slow" > $O/pytest_gpu_slow.log 2>&1
  ;;
term3)  # C4 terminal records at three rows per block (the compact image) against the cost model's two, ABAB
  timeout -k 10 300 python -u bench.py --no-e2e --no-probe --traffic off --rows-block 64:3 > $O/bench_c4_s3_parity.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu > $O/bench_c4_s2_1.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu --rows-block 64:3 > $O/bench_c4_s3_1.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu > $O/bench_c4_s2_2.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu --rows-block 64:3 > $O/bench_c4_s3_2.log 2>&1
  ;;
footprint)  # device bytes against the reference's RRR bytes at 100 M rows with the r06 defaults (terminal records)
  timeout -k 10 1100 python -u tools/footprint_scale.py > $O/footprint.jsonl 2> $O/footprint.log
  ;;
greedy_term_blocks)  # greedy + relax with terminal records (defaults) at the automatic block shape and 64:3 / 64:2
  timeout -k 10 900 python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0 --reps 10 --skip-small --blocks auto,64:3,64:2 > $O/greedy_term_blocks.log 2>&1
  ;;
prefetch)  # terminal walk reading the next field's words early: tests, then ABAB C4 and greedy against the previous build
  # (needs tools/_ab/libmbrwt_head.so: the previous commit's libmbrwt.so, copied there before the change)
  H="env MBRWT_LIB=tools/_ab/libmbrwt_head.so"
  timeout -k 10 400 $PYT tests/test_gpu_rows.py -k "terminal or async or errors or reference_grids or random_matrices or compact_cus" > $O/pytest_rows.log 2>&1 &&
  timeout -k 10 300 python -u bench.py --no-e2e --no-probe --traffic off > $O/bench_c4_parity.log 2>&1 &&
  timeout -k 10 200 $H $B --no-cpu > $O/bench_c4_head_1.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu > $O/bench_c4_new_1.log 2>&1 &&
  timeout -k 10 200 $H $B --no-cpu > $O/bench_c4_head_2.log 2>&1 &&
  timeout -k 10 200 $B --no-cpu > $O/bench_c4_new_2.log 2>&1 &&
  timeout -k 10 600 $H python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0 --reps 10 --skip-small > $O/greedy_head.log 2>&1 &&
  timeout -k 10 600 python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0 --reps 10 --skip-small > $O/greedy_new.log 2>&1
  ;;
c4_sq)  # SQ / TA counters of the C4 traversal with terminal records (r05's three passes)
  C="python -u bench.py --no-cpu --no-e2e --no-probe --traffic off --steps 3 --warmup 1"
  timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $O/sq1 -o run --output-format csv -- $C > $O/sq1.log 2>&1 &&
  timeout -s KILL 400 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $O/sq2 -o run --output-format csv -- $C > $O/sq2.log 2>&1 &&
  timeout -s KILL 400 rocprofv3 --pmc GRBM_COUNT GRBM_GUI_ACTIVE SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_WR TA_BUFFER_WAVEFRONTS_sum TA_TA_BUSY_sum -d $O/sq3 -o run --output-format csv -- $C > $O/sq3.log 2>&1
  ;;
configs)  # BASELINE configs[1] (C2) and configs[2] (C3) on HEAD: whole-batch parity, live PMC
  timeout -k 10 400 python -u bench.py --workload c2 --no-e2e > $O/bench_c2.log 2>&1 &&
  timeout -k 10 600 python -u bench.py --workload c3 --no-e2e > $O/bench_c3.log 2>&1
  ;;
c2ab)  # C2 (cache-resident) with terminal records against byte masks, ABAB
  timeout -k 10 200 $B --workload c2 --no-cpu --rows-code 3 > $O/bench_c2_byte_1.log 2>&1 &&
  timeout -k 10 200 $B --workload c2 --no-cpu > $O/bench_c2_term_1.log 2>&1 &&
  timeout -k 10 200 $B --workload c2 --no-cpu --rows-code 3 > $O/bench_c2_byte_2.log 2>&1 &&
  timeout -k 10 200 $B --workload c2 --no-cpu > $O/bench_c2_term_2.log 2>&1
  ;;
*) echo "unknown stage $STAGE"; exit 2 ;;
esac || exit $?
done
