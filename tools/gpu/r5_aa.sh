# r05 step AA: C3 lanes per row after the r04 unit split (G = 4 default vs 8 / 2)
set -o pipefail
O=gpurun_out/r5aa; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C3="--rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --steps 10 --warmup 3"
for r in 1 2; do
for g in 0 8 2; do
timeout -k 10 300 python -u tools/trav_ab.py $C3 --var-lanes $g --tag g${g}_$r > $O/c3_g${g}_$r.log 2>&1 || exit 1
done
done
