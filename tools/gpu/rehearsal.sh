# 2-rank rehearsal of the N>1 bench path on ONE GPU (gloo backend: RCCL needs one GPU per rank), smaller structure; then the N=1 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --rows 1000000000 --dist-backend gloo --no-cpu > gpurun_out/rehearsal.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
