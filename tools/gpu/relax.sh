# BRWTOptimizer::relax on the device: parity tests (Python + C++ mirror), then build+relax benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "relax or device_builder" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_relax.log 2>&1 || exit 1
timeout -k 10 300 tests/cpp/_build/test_brwt device > gpurun_out/cpp_brwt_device.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_build.py --arity 2 --relax 10 --reps 2 > gpurun_out/bench_relax_a2.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_build.py --arity 2 --reps 2 > gpurun_out/bench_build_a2.log 2>&1
