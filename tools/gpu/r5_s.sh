# r05 step S: footprint at 100 M rows against the reference's RRR bytes on
# the laws of its correlated generators, with and without record classes
set -o pipefail
O=gpurun_out/r5s; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1100 python -u tools/footprint_scale.py --cases uniform_rows:basic,iid:basic,weighted_rows:basic,uniform_rows:greedy,uniform_columns:basic,uniform_columns:greedy > $O/footprint.jsonl 2> $O/footprint.log || exit 1
