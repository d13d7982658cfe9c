set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/rows_ab.py --rows 3700000000 --batch 8000000 --steps 20 --configs "rows@+occ3+occ2+occ4+diag1.occ3+diag1.occ2" > gpurun_out/occ_c4.log 2>&1 || exit 1
