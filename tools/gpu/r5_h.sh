# r05 step H: dist / wire / row / shard tests after the build-option and
# two-stream changes; 2-rank rehearsal of bench.py's N > 1 step (gloo, one GPU)
set -o pipefail
O=gpurun_out/r5h; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dist.py tests/test_gpu_wire.py tests/test_gpu_rows.py tests/test_gpu_shards.py tests/test_gpu_files.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --dist-backend gloo --rows 1000000000 --steps 10 --warmup 3 --no-e2e > $O/rehearsal_2rank.log 2>&1 || exit 1
