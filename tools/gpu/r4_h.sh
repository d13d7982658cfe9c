# r04 step H: C3 variable-length decode at 6 waves per SIMD (79 VGPRs);
# labels stored from the walk (no LDS stage) vs the stage; SQ counters of both
set -o pipefail
mkdir -p gpurun_out/r4h
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py -k "variable" > gpurun_out/r4h/tests_var.log 2>&1 || exit 1
C3="--rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --steps 10 --configs rows@async"
for v in "1 4" "0 4" "0 8" "0 2"; do set -- $v
MBRWT_VAR_STAGE=$1 MBRWT_VAR_G=$2 timeout -k 10 240 python -u tools/rows_ab.py $C3 > gpurun_out/r4h/c3_s$1_g$2.log 2>&1 || exit 1
done
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH"
for st in 1 0; do
MBRWT_VAR_STAGE=$st MBRWT_VAR_G=4 timeout -s KILL 240 rocprofv3 --pmc $A --kernel-include-regex k_var_decode -d gpurun_out/r4h/sq_a_s$st -o run --output-format csv -- python tools/rows_ab.py --rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --steps 3 --configs rows@async > gpurun_out/r4h/sq_a_s$st.log 2>&1 || exit 1
MBRWT_VAR_STAGE=$st MBRWT_VAR_G=4 timeout -s KILL 240 rocprofv3 --pmc $B --kernel-include-regex k_var_decode -d gpurun_out/r4h/sq_b_s$st -o run --output-format csv -- python tools/rows_ab.py --rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --steps 3 --configs rows@async > gpurun_out/r4h/sq_b_s$st.log 2>&1 || exit 1
done
