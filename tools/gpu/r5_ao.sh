# r05 step AO: label regions of 768 instead of 1,024 per tile (denser temp
# region); row tests, then the bench step, order rel, a, a, rel (twice)
set -o pipefail
O=gpurun_out/r5ao; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py tests/test_gpu_classes.py > $O/tests.log 2>&1 || exit 1
A=tools/_ab/libmbrwt_c1024.so
BB="--steps 30 --warmup 5 --no-cpu --no-probe --traffic off --no-e2e"
for r in 1 2; do
timeout -k 10 300 python -u bench.py $BB > $O/bench_rel_a$r.log 2>&1 || exit 1
MBRWT_LIB=$A timeout -k 10 300 python -u bench.py $BB > $O/bench_c1024_b$r.log 2>&1 || exit 1
MBRWT_LIB=$A timeout -k 10 300 python -u bench.py $BB > $O/bench_c1024_c$r.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py $BB > $O/bench_rel_d$r.log 2>&1 || exit 1
done
