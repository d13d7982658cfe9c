# r05 step AK: non-temporal CSR stores in k_compact_tiles (release) vs plain
# (traversal stores non-temporal in both) vs all plain (r05 before these
# changes): the two-stream bench step, order rel, a, b, b, a, rel; row
# tests first
set -o pipefail
O=gpurun_out/r5ak; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py tests/test_gpu_classes.py tests/test_gpu_hostpipe.py > $O/tests.log 2>&1 || exit 1
A=tools/_ab/libmbrwt_plaincompact.so; B=tools/_ab/libmbrwt_plainall.so
BB="--steps 30 --warmup 5 --no-cpu --no-probe --traffic off --no-e2e"
for r in 1 2; do
timeout -k 10 300 python -u bench.py $BB > $O/bench_rel_a$r.log 2>&1 || exit 1
MBRWT_LIB=$A timeout -k 10 300 python -u bench.py $BB > $O/bench_plaincompact_b$r.log 2>&1 || exit 1
MBRWT_LIB=$B timeout -k 10 300 python -u bench.py $BB > $O/bench_plainall_c$r.log 2>&1 || exit 1
MBRWT_LIB=$B timeout -k 10 300 python -u bench.py $BB > $O/bench_plainall_d$r.log 2>&1 || exit 1
MBRWT_LIB=$A timeout -k 10 300 python -u bench.py $BB > $O/bench_plaincompact_e$r.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py $BB > $O/bench_rel_f$r.log 2>&1 || exit 1
done
