set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log | grep -q "pytest rc=0" || exit 1
timeout -k 10 600 python tools/sweep.py --variants 18 --reps 5 > gpurun_out/sweep_compact.log 2>&1
