set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/sweep.py --variants 5,10 --reps 5 > gpurun_out/sweep_nt.log 2>&1; echo "rc=$?" >> gpurun_out/sweep_nt.log
timeout -k 10 600 python tools/sweep.py --rows 1000000 --variants 4,5,10 --reps 5 > gpurun_out/sweep_c2.log 2>&1; echo "rc=$?" >> gpurun_out/sweep_c2.log
