# r05 step C: the rest of r5_b after the wide-unit test fix
set -o pipefail
O=gpurun_out/r5b; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rows.py -k "wide_units" tests/test_gpu_dist.py > $O/tests2.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/trav_ab.py --tag release > $O/trav_release.log 2>&1 || exit 1
for v in stamps nostore nt0; do
MBRWT_LIB=tools/_ab/libmbrwt_$v.so timeout -k 10 300 python -u tools/trav_ab.py --tag $v > $O/trav_$v.log 2>&1 || exit 1
done
timeout -k 10 600 python -u bench.py --traffic off > $O/bench.log 2>&1 || exit 1
