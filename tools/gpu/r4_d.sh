# r04 step D: the rest of the -m gpu suite (node-image kernels pinned to the
# nodes layout; C++ mirror, multi-device, wire, BinRel-WT on the defaults)
set -o pipefail
mkdir -p gpurun_out/r4d
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -v --maxfail=5 --timeout 300 --timeout-method thread -m "gpu and not slow" tests --deselect tests/test_gpu_rows.py --deselect tests/test_gpu_files.py --deselect tests/test_gpu_dist.py > gpurun_out/r4d/tests_rest.log 2>&1 || exit 1
