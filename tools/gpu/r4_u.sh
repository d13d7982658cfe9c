# r04 step U: bench.py two-stream step vs the events' cost and the step count
set -o pipefail
mkdir -p gpurun_out/r4u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python -u bench.py --no-cpu --traffic off --no-probe"
timeout -k 10 200 $B --steps 10 > gpurun_out/r4u/q2_all_s10.log 2>&1 || exit 1
timeout -k 10 200 $B --steps 10 --kernel-timing off > gpurun_out/r4u/q2_off_s10.log 2>&1 || exit 1
timeout -k 10 200 $B --steps 10 --kernel-timing first > gpurun_out/r4u/q2_first_s10.log 2>&1 || exit 1
timeout -k 10 200 $B --steps 40 > gpurun_out/r4u/q2_all_s40.log 2>&1 || exit 1
timeout -k 10 200 $B --steps 40 --kernel-timing off > gpurun_out/r4u/q2_off_s40.log 2>&1 || exit 1
timeout -k 10 200 $B --steps 10 --warmup 10 > gpurun_out/r4u/q2_all_s10_w10.log 2>&1 || exit 1
