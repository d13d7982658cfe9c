# r05 step AM: non-temporal CSR stores in the C3 variable-record decode vs
# plain; bench --workload c3 (two streams), order rel, nt, nt, rel
set -o pipefail
O=gpurun_out/r5am; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A=tools/_ab/libmbrwt_varnt.so
BB="--workload c3 --steps 20 --warmup 5 --no-cpu --no-probe --traffic off --no-e2e"
timeout -k 10 400 python -u bench.py $BB > $O/bench_rel_a.log 2>&1 || exit 1
MBRWT_LIB=$A timeout -k 10 400 python -u bench.py $BB > $O/bench_nt_b.log 2>&1 || exit 1
MBRWT_LIB=$A timeout -k 10 400 python -u bench.py $BB > $O/bench_nt_c.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py $BB > $O/bench_rel_d.log 2>&1 || exit 1
