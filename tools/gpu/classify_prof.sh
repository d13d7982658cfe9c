# per-dispatch durations of the classify kernels (raw trace in /tmp, filtered rows copied)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/pt -o run --output-format csv -- python tools/bench_classify.py --top 10 --steps 3 > gpurun_out/cls_prof_top.log 2>&1 || exit 1
f=$(find /tmp/pt -name "*kernel_trace.csv" | head -1)
head -1 "$f" > gpurun_out/cls_top_trace.csv
grep -E "read_top_labels|read_labels|traverse_fast2|compact_chunks" "$f" >> gpurun_out/cls_top_trace.csv
