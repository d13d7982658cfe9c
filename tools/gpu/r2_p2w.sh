# round 2: k_traverse_p2w correctness (GPU parity tests) and A/B of its configurations
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/sweep.py --variants ${C4V:-17,20,21,22,23} --reps 5 > gpurun_out/sweep_c4.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/sweep.py --rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --variants ${C3V:-17,20,21,22,23} --reps 3 > gpurun_out/sweep_c3.log 2>&1
