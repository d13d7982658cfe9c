set -o pipefail
mkdir -p gpurun_out/st2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MBRWT_ROWS_STAGE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rows.py > gpurun_out/st2/tests_stage.log 2>&1 || exit 1
timeout -k 10 200 python tools/rows_ab.py --rows 3700000000 --batch 8000000 --steps 20 --configs "rows@async+stage.async+stage.occ4.async" > gpurun_out/st2/c4.log 2>&1 || exit 1
timeout -k 10 100 python tools/rows_ab.py --rows 1000000 --batch 1000000 --steps 50 --configs "rows@async+stage.async" > gpurun_out/st2/c2.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "beyond_2_32" > gpurun_out/st2/tests_builder_2_32.log 2>&1 || exit 1
