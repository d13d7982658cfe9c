# r05 step AD: how much the C4 traversal depends on its resident waves --
# 24 per CU (release: three 8-wave workgroups) against 16 (an A/B build whose
# launch asks 1 KB more LDS per workgroup: two fit), same box, 3 rounds
set -o pipefail
O=gpurun_out/r5ad; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
timeout -k 10 300 python -u tools/trav_ab.py --tag rel$r > $O/c4_rel_$r.log 2>&1 || exit 1
MBRWT_LIB=tools/_ab/libmbrwt_ldspad.so timeout -k 10 300 python -u tools/trav_ab.py --tag w16_$r > $O/c4_w16_$r.log 2>&1 || exit 1
done
