# r04 step Y: 2-rank rehearsal of bench.py's N > 1 step on one GPU over gloo
# (the device-sized wire with the r04 pack / unpack / offsets kernels;
# whole-global-batch parity on rank 0), 1 B rows to fit two images
set -o pipefail
mkdir -p gpurun_out/r4y
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --rows 1000000000 --steps 10 --warmup 3 > gpurun_out/r4y/rehearsal_2rank_gloo.log 2>&1 || exit 1
