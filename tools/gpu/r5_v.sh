# r05 step V: the -m gpu suite without the slow cases on the final sources (record
# classes, the class lookup in the traversal), smoke.  A
# heartbeat line per minute keeps the run visibly alive through long cases
# (pytest's own per-test timeout bounds a hang).
set -o pipefail
O=gpurun_out/r5v; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( for i in $(seq 1 20); do sleep 60; echo "heartbeat $i $(date +%T)" >> $O/heartbeat.log; done ) &
HB=$!
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m "gpu and not slow" tests > $O/pytest_gpu_not_slow.log 2>&1
rc=$?
kill $HB 2>/dev/null
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
