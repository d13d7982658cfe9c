# r05 step R: record classes (csrc/rows_class.hip) -- their GPU parity, the
# row-record suite after the record-reader header move, C4 unchanged (AUTO
# samples and declines)
set -o pipefail
O=gpurun_out/r5r; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_classes.py tests/test_gpu_rows.py -k "block_shape or classes" > $O/tests_classes.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py tests/test_gpu_files.py > $O/tests_rows.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/trav_ab.py --tag c4 > $O/c4.log 2>&1 || exit 1
