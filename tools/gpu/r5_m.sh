# r05 step M: long records walked from an LDS copy in the traversal; C3 decode
# with word-wise mask reads and paired label stores -- row tests, C3 timing
# and SQ counters, greedy at 3.7 B, C4
set -o pipefail
O=gpurun_out/r5m; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py tests/test_gpu_files.py > $O/tests.log 2>&1 || exit 1
C3="--rows 1000000000 --cols 3173 --density 0.038 --batch 10000000"
timeout -k 10 400 python -u tools/trav_ab.py $C3 --steps 10 --warmup 3 --tag c3 > $O/c3.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAVES --kernel-include-regex k_var_decode -d $O/c3_sq -o run --output-format csv -- python tools/trav_ab.py $C3 --steps 3 --warmup 2 --tag sq > $O/c3_sq.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0 --reps 20 --skip-small > $O/greedy_3p7B.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/trav_ab.py --tag c4 > $O/c4.log 2>&1 || exit 1
