# 4-ary wavelet matrix: BinRel-WT parity tests, then the C5 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_binrel_wt.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_wt.log 2>&1 || exit 1
timeout -k 10 900 python -u tools/bench_binrel_wt.py > gpurun_out/wt_c5_bench.log 2>&1
