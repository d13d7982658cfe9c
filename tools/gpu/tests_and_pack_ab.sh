set -o pipefail
mkdir -p gpurun_out
make -s -C tests/cpp > gpurun_out/cpp_build.log 2>&1
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log | grep -q "pytest rc=0" || exit 1
timeout -k 10 600 python tools/sweep.py --variants 18 --reps 5 > gpurun_out/sweep_pack.log 2>&1 || exit 1
MBRWT_PACK=0 timeout -k 10 600 python tools/sweep.py --variants 18 --reps 5 > gpurun_out/sweep_nopack.log 2>&1 || exit 1
timeout -k 10 600 python tools/sweep.py --rows 1000000 --variants 17 --reps 5 > gpurun_out/sweep_pack_c2.log 2>&1
