# r05 step AJ: whole lines + non-temporal temp stores (release) vs
# non-temporal with the partly written last line vs whole lines with plain
# stores; row tests first; order rel, a, b, b, a, rel (twice); then bench
set -o pipefail
O=gpurun_out/r5aj; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py tests/test_gpu_classes.py > $O/tests.log 2>&1 || exit 1
A=tools/_ab/libmbrwt_ntpartial.so; B=tools/_ab/libmbrwt_fullplain.so
for r in 1 2; do
timeout -k 10 300 python -u tools/trav_ab.py --tag relA$r > $O/c4_rel_a$r.log 2>&1 || exit 1
MBRWT_LIB=$A timeout -k 10 300 python -u tools/trav_ab.py --tag ntpB$r > $O/c4_ntpartial_b$r.log 2>&1 || exit 1
MBRWT_LIB=$B timeout -k 10 300 python -u tools/trav_ab.py --tag fpC$r > $O/c4_fullplain_c$r.log 2>&1 || exit 1
MBRWT_LIB=$B timeout -k 10 300 python -u tools/trav_ab.py --tag fpD$r > $O/c4_fullplain_d$r.log 2>&1 || exit 1
MBRWT_LIB=$A timeout -k 10 300 python -u tools/trav_ab.py --tag ntpE$r > $O/c4_ntpartial_e$r.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/trav_ab.py --tag relF$r > $O/c4_rel_f$r.log 2>&1 || exit 1
done
timeout -k 10 600 python -u bench.py --no-cpu > $O/bench_c4.log 2>&1 || exit 1
