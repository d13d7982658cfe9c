# round 2: full-size parity of C3 (Multi-BRWT 1B x 3,173) and C5 (BinRel-WT 1B x 3,173)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest tests/test_full_size.py -m gpu -x -v -s --timeout 900 --timeout-method thread > gpurun_out/pytest_full_size.log 2>&1
