# r04 step M: which streams overlap (two pool streams vs the null stream +
# a pool stream), bench.py --query-streams 2 with the whole-batch parity
set -o pipefail
mkdir -p gpurun_out/r4m
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/overlap_ab.py --steps 40 > gpurun_out/r4m/overlap.log 2>&1 || exit 1
timeout -k 10 500 python -u bench.py --traffic off --steps 30 --query-streams 2 > gpurun_out/r4m/bench_q2_parity.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py -k "variable" > gpurun_out/r4m/tests_var.log 2>&1 || exit 1
C3="--rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --steps 10 --configs rows@async"
for g in 8 4 8; do
MBRWT_VAR_G=$g timeout -k 10 240 python -u tools/rows_ab.py $C3 >> gpurun_out/r4m/c3_g$g.log 2>&1 || exit 1
done
