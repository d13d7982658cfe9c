# r05 step F: is the C4 traversal bound by its request pattern or by its
# work?  Block loads only (registers / LDS staging), persistent and
# one-tile-per-wave grids, beside the random-request probe on this box
set -o pipefail
O=gpurun_out/r5f; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u tools/trav_ab.py --tag release --probe > $O/trav_release.log 2>&1 || exit 1
for v in gather gather_tpw1 loadonly loadonly_tpw1 tpw1; do
MBRWT_LIB=tools/_ab/libmbrwt_$v.so timeout -k 10 300 python -u tools/trav_ab.py --tag $v > $O/trav_$v.log 2>&1 || exit 1
done
