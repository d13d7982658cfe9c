# r04 step X: refresh the README's other configs on the final sources: C2
# (bench.py --workload c2) and 4.5 B rows in one row-record image (u64 rows)
set -o pipefail
mkdir -p gpurun_out/r4x
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py --workload c2 --traffic off > gpurun_out/r4x/bench_c2.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/rows_ab.py --rows 4500000000 --batch 8000000 --steps 30 --configs "rows@async" --oracle > gpurun_out/r4x/rows_4p5B.log 2>&1 || exit 1
