set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_binrel_wt.py -x -q > gpurun_out/pytest_wt.log 2>&1 || exit 1
timeout -k 10 600 python tools/bench_binrel_wt.py --rows 100000000 --batch 2000000 > gpurun_out/bench_wt_100m.log 2>&1 || exit 1
timeout -k 10 900 python tools/bench_binrel_wt.py > gpurun_out/bench_wt_full.log 2>&1
