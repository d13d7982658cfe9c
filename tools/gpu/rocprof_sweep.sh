set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sweep -o run --output-format csv -- python tools/sweep.py --variants 18 --reps 5 > gpurun_out/prof_sweep.log 2>&1
