# r04 step N: C3 decode with 8 lanes per row at 24 waves per CU (79 VGPRs)
# against 4 lanes per row (16 waves, LDS-bound); the VAR tests
set -o pipefail
mkdir -p gpurun_out/r4n
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py -k "variable" > gpurun_out/r4n/tests_var.log 2>&1 || exit 1
C3="--rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --steps 10 --configs rows@async"
for g in 8 4 8; do
MBRWT_VAR_G=$g timeout -k 10 240 python -u tools/rows_ab.py $C3 >> gpurun_out/r4n/c3_g$g.log 2>&1 || exit 1
done
