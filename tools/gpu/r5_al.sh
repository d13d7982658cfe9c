# r05 step AL: non-temporal loads of the data read once (row ids, spill
# entries, the compaction's temp reads) vs the release; bench step and
# kernel, order rel, nt, nt, rel (twice)
set -o pipefail
O=gpurun_out/r5al; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A=tools/_ab/libmbrwt_ntloads.so
BB="--steps 30 --warmup 5 --no-cpu --no-probe --traffic off --no-e2e"
for r in 1 2; do
timeout -k 10 300 python -u bench.py $BB > $O/bench_rel_a$r.log 2>&1 || exit 1
MBRWT_LIB=$A timeout -k 10 300 python -u bench.py $BB > $O/bench_ntl_b$r.log 2>&1 || exit 1
MBRWT_LIB=$A timeout -k 10 300 python -u bench.py $BB > $O/bench_ntl_c$r.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py $BB > $O/bench_rel_d$r.log 2>&1 || exit 1
done
