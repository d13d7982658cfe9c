# PACK2 layout: parity tests, then same-box A/B of the Kingsford-shape traversal (PACK2 vs PACK-only)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "pack" --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/sweep.py --variants 0 --reps 5 > gpurun_out/sweep_pack2.log 2>&1 || exit 1
MBRWT_PACK2=0 timeout -k 10 300 python -u tools/sweep.py --variants 0 --reps 5 > gpurun_out/sweep_pack1.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/sweep.py --rows 1000000 --variants 0 --reps 5 > gpurun_out/sweep_pack2_c2.log 2>&1
