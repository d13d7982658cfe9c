set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/sweep.py --variants 4,5 --fold 0,1 --reps 5 > gpurun_out/sweep_fold.log 2>&1; echo "rc=$?" >> gpurun_out/sweep_fold.log
