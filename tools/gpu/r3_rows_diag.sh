# v2 row-record kernel: where the time goes (diagnostic variants, WRONG results
# by design) at C4, plus a kernel trace of two C2 contexts (step overhead)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/rows_ab.py --rows 3700000000 --batch 8000000 --configs "rows@+diag1+diag2+diag4+diag5+diag7" > gpurun_out/diag_c4.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_c2 -o run --output-format csv -- python tools/rows_ab.py --rows 1000000 --batch 1000000 --configs "rows;rows:64,2;rows:128,4" > gpurun_out/kt_c2.log 2>&1 || exit 1
