set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/sweep.py --variants 18,21 --reps 5 > gpurun_out/sweep_diag.log 2>&1 || exit 1
timeout -k 10 600 python tools/sweep.py --rows 1000000 --variants 17,21 --reps 5 > gpurun_out/sweep_diag_c2.log 2>&1
