# round 2 (final A): the whole GPU suite, then the default bench (live PMC traffic, CPU legs)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1 &&
timeout -k 10 540 python -u bench.py --traffic-out gpurun_out/traffic_c4.json > gpurun_out/bench.log 2>&1
