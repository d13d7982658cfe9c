# r05 step Q: same-box C4 A/B -- 24-bit vs 32-bit multiplies in the path
# walk, and the persistent grid, three rounds interleaved
set -o pipefail
O=gpurun_out/r5q; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
timeout -k 10 300 python -u tools/trav_ab.py --tag rel$r > $O/c4_rel_$r.log 2>&1 || exit 1
MBRWT_LIB=tools/_ab/libmbrwt_mul32.so timeout -k 10 300 python -u tools/trav_ab.py --tag mul32_$r > $O/c4_mul32_$r.log 2>&1 || exit 1
done
