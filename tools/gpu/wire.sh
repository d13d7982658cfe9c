# bit-packed all-gatherv: GPU kernel test, 2-rank gloo rehearsal (CUDA tensors -> HIP pack/unpack), full GPU suite
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k pack_ids -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_wire.log 2>&1 || exit 1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --rows 1000000000 --dist-backend gloo --no-cpu > gpurun_out/rehearsal.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
