# r05 step T: the class lookup inside k_traverse_rows (no separate map
# launch): class tests, C4 unchanged, footprint at 100 M rows again
set -o pipefail
O=gpurun_out/r5t; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_classes.py > $O/tests_classes.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/trav_ab.py --tag c4 > $O/c4.log 2>&1 || exit 1
timeout -k 10 900 python -u tools/footprint_scale.py --cases uniform_rows:basic,weighted_rows:basic,uniform_rows:greedy,uniform_columns:basic,uniform_columns:greedy > $O/footprint.jsonl 2> $O/footprint.log || exit 1
