# r05 step I: one tile per wave (k_traverse_rows, k_var_decode) and computed
# unit bases in the variable-record decode -- row tests; C4 and C3 A/B
set -o pipefail
O=gpurun_out/r5i; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py tests/test_gpu_hostpipe.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/trav_ab.py --tag release > $O/c4_release.log 2>&1 || exit 1
MBRWT_LIB=tools/_ab/libmbrwt_persistent.so timeout -k 10 300 python -u tools/trav_ab.py --tag persistent > $O/c4_persistent.log 2>&1 || exit 1
C3="--rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --steps 10 --warmup 3"
timeout -k 10 400 python -u tools/trav_ab.py $C3 --tag release > $O/c3_release.log 2>&1 || exit 1
for v in persistent nous; do
MBRWT_LIB=tools/_ab/libmbrwt_$v.so timeout -k 10 400 python -u tools/trav_ab.py $C3 --tag $v > $O/c3_$v.log 2>&1 || exit 1
done
timeout -k 10 500 python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0 --reps 20 --skip-small > $O/greedy_3p7B.log 2>&1 || exit 1
