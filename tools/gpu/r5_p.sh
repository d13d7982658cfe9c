# r05 step P: full-rate multiplies (a shift for the unit bases at C3, 24-bit
# multiplies in the path walk at C4); row tests; C3 and C4 timing
set -o pipefail
O=gpurun_out/r5p; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/trav_ab.py --rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --steps 10 --warmup 3 --tag c3 > $O/c3.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/trav_ab.py --tag c4 > $O/c4.log 2>&1 || exit 1
