# r05 step W: the slow full-size -m gpu cases on the final sources (C3, C4,
# C5 at full size, rows >= 2^32), heartbeat per minute
set -o pipefail
O=gpurun_out/r5w; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( for i in $(seq 1 20); do sleep 60; echo "heartbeat $i $(date +%T)" >> $O/heartbeat.log; done ) &
HB=$!
timeout -k 10 1100 python -u -m pytest -v --timeout 600 --timeout-method thread -m "gpu and slow" tests > $O/pytest_gpu_slow.log 2>&1
rc=$?
kill $HB 2>/dev/null
exit $rc
