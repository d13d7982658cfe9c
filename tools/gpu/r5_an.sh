# r05 step AN: 2-rank rehearsal of bench.py's N > 1 step on the final sources
# (gloo, both ranks on one GPU, 1 B rows so two images fit)
set -o pipefail
O=gpurun_out/r5an; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --dist-backend gloo --rows 1000000000 --steps 10 --warmup 3 --no-e2e > $O/rehearsal_2rank.log 2>&1 || exit 1
