# r05 step Z: the path walk's 24-bit mads named (v_mad_u32_u24) instead of
# the compiler's 64-bit fold, and the leaf parent's column computed on a
# linear path table -- odometer tests, same-box C4 A/B (release / nolin /
# neither), 3 rounds
set -o pipefail
O=gpurun_out/r5z; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py -k "odometer or synthetic_c2 or ranged or every_block or reference_grids" > $O/tests.log 2>&1 || exit 1
for r in 1 2 3; do
timeout -k 10 300 python -u tools/trav_ab.py --tag rel$r > $O/c4_rel_$r.log 2>&1 || exit 1
MBRWT_LIB=tools/_ab/libmbrwt_nolin.so timeout -k 10 300 python -u tools/trav_ab.py --tag nolin$r > $O/c4_nolin_$r.log 2>&1 || exit 1
MBRWT_LIB=tools/_ab/libmbrwt_noasm24.so timeout -k 10 300 python -u tools/trav_ab.py --tag noasm$r > $O/c4_noasm_$r.log 2>&1 || exit 1
done
