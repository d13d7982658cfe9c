# SQ counter passes (one rocprofv3 --pmc run per pass) of k_traverse_rows at the
# Kingsford shape (400 M rows, 8 M-row batch), plus a kernel trace of two C2
# contexts (step-overhead check)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_c2 -o run --output-format csv -- python tools/rows_ab.py --rows 1000000 --batch 1000000 --configs "rows;rows:64,2" > gpurun_out/kt_c2.log 2>&1 || exit 1
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_BRANCH"
P2="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex k_traverse_rows -d gpurun_out/sq_$i -o run --output-format csv -- python tools/rows_ab.py --rows 400000000 --batch 8000000 --steps 3 --configs rows > gpurun_out/sq_$i.log 2>&1 || exit 1
done
