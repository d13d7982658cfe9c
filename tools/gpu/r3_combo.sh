set -o pipefail
mkdir -p gpurun_out/v4 gpurun_out/greedy
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 ./tools/_build/glds_exec_probe > gpurun_out/v4/glds_exec_probe.json 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "greedy_builder" > gpurun_out/greedy/tests.log 2>&1 || exit 1
MBRWT_ROWS_KERNEL=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py > gpurun_out/v4/tests_v4.log 2>&1
timeout -k 10 200 python tools/rows_ab.py --rows 3700000000 --batch 8000000 --steps 20 --configs "rows@async+v4.async+split.async" > gpurun_out/v4/c4.log 2>&1 || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 2 --rows 1000000000 --dist-backend gloo --no-cpu --no-probe --traffic off > gpurun_out/v4/rehearsal_2rank_gloo_devwire.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/sweep.py --rows 1000000000 --cols 3173 --density 0.038 --batch 10000000 --variants 0,20 --reps 10 > gpurun_out/v4/c3_sweep.log 2>&1 || exit 1
