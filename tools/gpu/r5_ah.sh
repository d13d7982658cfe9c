# r05 step AH: do the traversal's own stores slow its block loads? The final
# kernel against an A/B build without the temp-region stores, ABBA order
set -o pipefail
O=gpurun_out/r5ah; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NS=tools/_ab/libmbrwt_nostore.so
for r in 1 2; do
timeout -k 10 300 python -u tools/trav_ab.py --tag relA$r > $O/c4_relA_$r.log 2>&1 || exit 1
MBRWT_LIB=$NS timeout -k 10 300 python -u tools/trav_ab.py --tag nsB$r > $O/c4_nsB_$r.log 2>&1 || exit 1
MBRWT_LIB=$NS timeout -k 10 300 python -u tools/trav_ab.py --tag nsC$r > $O/c4_nsC_$r.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/trav_ab.py --tag relD$r > $O/c4_relD_$r.log 2>&1 || exit 1
done
