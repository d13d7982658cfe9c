# r05 step D: dynamic tile claims in k_traverse_rows, DPP scans, the
# pipelined host path, the variable-record LDS bound: row / hostpipe / dist
# tests; C4 A/B (claims vs the static order, with per-wave stamps; no temp
# stores); bench with the end-to-end leg
set -o pipefail
O=gpurun_out/r5d; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dist.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/trav_ab.py --tag release > $O/trav_release.log 2>&1 || exit 1
for v in static stamps static_stamps nostore; do
MBRWT_LIB=tools/_ab/libmbrwt_$v.so timeout -k 10 300 python -u tools/trav_ab.py --tag $v --stamps-out $O/stamps_$v.npy > $O/trav_$v.log 2>&1 || exit 1
done
timeout -k 10 600 python -u bench.py --traffic off > $O/bench.log 2>&1 || exit 1
