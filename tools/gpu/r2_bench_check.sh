# round 2: new GPU tests, the C++ mirror on the device, a small bench (live PMC traffic), a 2-rank
# strong-scaling rehearsal on one GPU (gloo), then the default bench
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "two_streams or null_cols or top_labels" > gpurun_out/pytest_new.log 2>&1 || exit 1
timeout -k 10 120 tests/cpp/_build/test_annotation device > gpurun_out/cpp_annotation_device.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --rows 200000000 --batch 1000000 --steps 3 --traffic-out gpurun_out/traffic_small.json > gpurun_out/bench_small.log 2>&1 || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --rows 200000000 --batch 2000000 --dist-backend gloo --no-probe > gpurun_out/rehearsal.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --traffic-out gpurun_out/traffic_c4.json > gpurun_out/bench.log 2>&1
