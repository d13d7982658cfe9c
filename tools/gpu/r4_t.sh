# r04 step T: which stream combinations overlap consecutive batches (2 and 3
# query contexts; default / pool / high-priority streams)
set -o pipefail
mkdir -p gpurun_out/r4t
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u tools/overlap_ab.py --steps 40 > gpurun_out/r4t/overlap.log 2>&1 || exit 1
