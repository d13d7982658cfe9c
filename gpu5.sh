set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log | grep -q "pytest rc=0" || exit 1
timeout -k 10 400 python tools/sweep.py --variants 3,4,5 > gpurun_out/sweep.log 2>&1; echo "rc=$?" >> gpurun_out/sweep.log
