set -o pipefail
mkdir -p gpurun_out
make -s -C tests/cpp > gpurun_out/cpp_build.log 2>&1
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
