set -o pipefail
mkdir -p gpurun_out/sc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/rows_ab.py --rows 4500000000 --batch 8000000 --steps 20 --oracle --configs "rows@async" > gpurun_out/sc/rows_4p5B_oracle.log 2>&1 || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 2 --rows 1000000000 --dist-backend gloo --no-cpu --no-probe --traffic off > gpurun_out/sc/rehearsal_2rank_gloo.log 2>&1 || exit 1
timeout -k 10 420 python -u bench.py --workload c3 --no-cpu --traffic-out gpurun_out/sc/c3_traffic.json > gpurun_out/sc/bench_c3.log 2>&1 || exit 1
