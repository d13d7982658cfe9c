# r05 step U: C3 stage readback as 8-byte LDS reads -- variable-record
# tests, same-box A/B against the four u16 reads (MBRWT_AB_STAGE16), and the
# LDS counters of the new decode
set -o pipefail
O=gpurun_out/r5u; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py -k "variable" > $O/tests.log 2>&1 || exit 1
C3="--rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --steps 10 --warmup 3"
for r in 1 2; do
timeout -k 10 300 python -u tools/trav_ab.py $C3 --tag rel$r > $O/c3_rel_$r.log 2>&1 || exit 1
MBRWT_LIB=tools/_ab/libmbrwt_stage16.so timeout -k 10 300 python -u tools/trav_ab.py $C3 --tag s16_$r > $O/c3_s16_$r.log 2>&1 || exit 1
done
C3S="--rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --steps 3 --warmup 2"
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS --kernel-include-regex k_var_decode -d $O/c3_sq -o run --output-format csv -- python tools/trav_ab.py $C3S --tag sq > $O/c3_sq.log 2>&1 || exit 1
