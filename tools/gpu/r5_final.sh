# r05 final check on the final sources: the -m gpu suite (not slow), smoke,
# bench C4 (live PMC, ceilings, CPU baseline, end-to-end, whole-batch parity)
# and its kernel trace; heartbeat per minute
set -o pipefail
O=gpurun_out/r5final2; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( for i in $(seq 1 25); do sleep 60; echo "heartbeat $i $(date +%T)" >> $O/heartbeat.log; done ) &
HB=$!
timeout -k 10 800 python -u -m pytest -v --timeout 300 --timeout-method thread -m "gpu and not slow" tests > $O/pytest_gpu_not_slow.log 2>&1
rc=$?
[ $rc -eq 0 ] || { kill $HB 2>/dev/null; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { kill $HB 2>/dev/null; exit 1; }
timeout -k 10 600 python -u bench.py --traffic-out $O/traffic_c4.json > $O/bench_c4.log 2>&1 || { kill $HB 2>/dev/null; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run --output-format csv -- python -u bench.py --no-cpu --no-e2e --no-probe --traffic off > $O/bench_c4_under_rocprof.log 2>&1
rc=$?
kill $HB 2>/dev/null
exit $rc
