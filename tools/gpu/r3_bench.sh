set -o pipefail
mkdir -p gpurun_out/r3b
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u bench.py --traffic-out gpurun_out/r3b/traffic.json > gpurun_out/r3b/bench.log 2>&1 || exit 1
