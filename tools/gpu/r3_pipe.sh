set -o pipefail
mkdir -p gpurun_out/pipe
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 3 --rows 1000000000 --dist-backend gloo --no-cpu --no-probe --traffic off > gpurun_out/pipe/rehearsal_2rank_gloo.log 2>&1 || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --steps 6 --warmup 2 --rows 100000000 --batch 1000000 --dist-backend gloo --check-rows 1000000 --cpu-sample 2000 --cpu-sample-1t 200 --no-probe --traffic off > gpurun_out/pipe/rehearsal_2rank_gloo_parity.log 2>&1 || exit 1
