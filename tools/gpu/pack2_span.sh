# PACK2 with per-node span: parity tests, then Kingsford (C4) and RefSeq (C3) sweeps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/sweep.py --variants 0 --reps 5 > gpurun_out/sweep_c4.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/sweep.py --rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --variants 0 --reps 3 > gpurun_out/sweep_c3.log 2>&1
