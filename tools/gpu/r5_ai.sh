# r05 step AI: the traversal's temp-region stores -- whole 128-byte lines
# (release) vs the old partly written last line vs non-temporal stores;
# row tests first; order rel, partial, nt, nt, partial, rel (twice)
set -o pipefail
O=gpurun_out/r5ai; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py tests/test_gpu_classes.py > $O/tests.log 2>&1 || exit 1
PA=tools/_ab/libmbrwt_partial.so; NT=tools/_ab/libmbrwt_ntstore.so
for r in 1 2; do
timeout -k 10 300 python -u tools/trav_ab.py --tag relA$r > $O/c4_rel_a$r.log 2>&1 || exit 1
MBRWT_LIB=$PA timeout -k 10 300 python -u tools/trav_ab.py --tag paB$r > $O/c4_partial_b$r.log 2>&1 || exit 1
MBRWT_LIB=$NT timeout -k 10 300 python -u tools/trav_ab.py --tag ntC$r > $O/c4_nt_c$r.log 2>&1 || exit 1
MBRWT_LIB=$NT timeout -k 10 300 python -u tools/trav_ab.py --tag ntD$r > $O/c4_nt_d$r.log 2>&1 || exit 1
MBRWT_LIB=$PA timeout -k 10 300 python -u tools/trav_ab.py --tag paE$r > $O/c4_partial_e$r.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/trav_ab.py --tag relF$r > $O/c4_rel_f$r.log 2>&1 || exit 1
done
