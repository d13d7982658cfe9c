set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log | grep -q "pytest rc=0" || exit 1
timeout -k 10 600 python tools/sweep.py --rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --variants 18 --reps 3 > gpurun_out/sweep_c3_pack.log 2>&1 || exit 1
MBRWT_PACK=0 timeout -k 10 600 python tools/sweep.py --rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --variants 18 --reps 3 > gpurun_out/sweep_c3_nopack.log 2>&1
