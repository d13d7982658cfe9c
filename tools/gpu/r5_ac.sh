# r05 step AC: the slow full-size cases and the greedy + relax shape at 3.7 B
# rows (whole batch against the streamed shaped oracle) on the final sources
set -o pipefail
O=gpurun_out/r5ac2; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( for i in $(seq 1 20); do sleep 60; echo "heartbeat $i $(date +%T)" >> $O/heartbeat.log; done ) &
HB=$!
timeout -k 10 700 python -u -m pytest -v --timeout 600 --timeout-method thread -m "gpu and slow" tests > $O/pytest_gpu_slow.log 2>&1
rc=$?
[ $rc -eq 0 ] || { kill $HB 2>/dev/null; exit $rc; }
timeout -k 10 400 python -u tools/bench_greedy.py --shape-npz tools/data/greedy_relax10_c2_shape.npz --scaled-rows 3700000000 --layout rows --variants 0 --reps 10 --skip-small > $O/greedy_3p7B.log 2>&1
rc=$?
kill $HB 2>/dev/null
exit $rc
