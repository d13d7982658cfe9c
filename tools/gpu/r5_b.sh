# r05 step B: DPP wave scans (traversal + compaction), the pipelined host
# path, the variable-record LDS bound -- row / hostpipe / wire tests; C4 A/B
# (release, stamps, no temp stores, plain loads); bench with the e2e leg
set -o pipefail
O=gpurun_out/r5b; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_hostpipe.py tests/test_gpu_rows.py tests/test_gpu_dist.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/trav_ab.py --tag release > $O/trav_release.log 2>&1 || exit 1
for v in stamps nostore nt0; do
MBRWT_LIB=tools/_ab/libmbrwt_$v.so timeout -k 10 300 python -u tools/trav_ab.py --tag $v > $O/trav_$v.log 2>&1 || exit 1
done
timeout -k 10 600 python -u bench.py --traffic off > $O/bench.log 2>&1 || exit 1
