# r04 step L: same-box A/B of the C4 step across this round's commits
# (6bf1e26: before the tree odometer; 02ea363: tree odometer; current:
# leaf-parent column lists, per-row long records, compaction stack sized by
# height), then batch k+1 on a clone's stream while batch k finishes
set -o pipefail
mkdir -p gpurun_out/r4l
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rows.py -k clone > gpurun_out/r4l/tests_clone.log 2>&1 || exit 1
C4="--rows 3700000000 --batch 8000000 --steps 30 --configs rows@async"
timeout -k 10 200 python -u tools/rows_ab.py $C4 > gpurun_out/r4l/c4_cur1.log 2>&1 || exit 1
MBRWT_LIB=tools/_ab/libmbrwt_6bf1e26.so timeout -k 10 200 python -u tools/rows_ab.py $C4 > gpurun_out/r4l/c4_6bf1e26.log 2>&1 || exit 1
MBRWT_LIB=tools/_ab/libmbrwt_02ea363.so timeout -k 10 200 python -u tools/rows_ab.py $C4 > gpurun_out/r4l/c4_02ea363.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/rows_ab.py $C4 > gpurun_out/r4l/c4_cur2.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/overlap_ab.py --steps 40 > gpurun_out/r4l/overlap.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu --traffic off --steps 30 --query-streams 2 > gpurun_out/r4l/bench_q2.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu --traffic off --steps 30 --query-streams 1 > gpurun_out/r4l/bench_q1.log 2>&1 || exit 1
