set -o pipefail
mkdir -p gpurun_out/fp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u tools/footprint.py > gpurun_out/fp/footprint.log 2>&1 || exit 1
