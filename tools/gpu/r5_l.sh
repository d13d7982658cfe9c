# r05 step L: where the greedy + relax step goes (kernel trace); SQ counters
# of the C3 variable-record decode (LDS bank conflicts)
set -o pipefail
O=gpurun_out/r5l; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/greedy_trace -o run --output-format csv -- python tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0 --reps 10 --skip-small > $O/greedy_trace.log 2>&1 || exit 1
C3="--rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --steps 3 --warmup 2"
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH"
i=0
for P in "$A" "$B"; do i=$((i+1))
timeout -s KILL 300 rocprofv3 --pmc $P --kernel-include-regex k_var_decode -d $O/c3_sq$i -o run --output-format csv -- python tools/trav_ab.py $C3 --tag sq$i > $O/c3_sq$i.log 2>&1 || exit 1
done
