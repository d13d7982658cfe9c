# r04 step F: C3 variable-length decode, lanes per row A/B (G = 1, 2, 4)
set -o pipefail
mkdir -p gpurun_out/r4f
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for g in 2 1 4; do
MBRWT_VAR_G=$g timeout -k 10 240 python -u tools/rows_ab.py --rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --steps 10 --configs "rows@async" > gpurun_out/r4f/c3_g$g.log 2>&1 || exit 1
done
