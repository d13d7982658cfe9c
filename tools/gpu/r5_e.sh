# r05 step E: balancing the persistent traversal's waves -- non-persistent
# grids (1 / 2 / 4 tiles per wave), issue priority for the later-dispatched
# workgroups; same-box C4 A/B with per-wave stamps
set -o pipefail
O=gpurun_out/r5e; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/trav_ab.py --tag release > $O/trav_release.log 2>&1 || exit 1
for v in tpw1 tpw2 tpw4 prio stamps tpw2_stamps prio_stamps; do
MBRWT_LIB=tools/_ab/libmbrwt_$v.so timeout -k 10 300 python -u tools/trav_ab.py --tag $v --stamps-out $O/stamps_$v.npy > $O/trav_$v.log 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/trav_ab.py --tag release2 > $O/trav_release2.log 2>&1 || exit 1
