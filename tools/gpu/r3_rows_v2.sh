# row-record kernel v2: parity tests, v1/v2 A/B at C2 and C4, SQ counters of v2
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rows.py -k "not beyond" > gpurun_out/rows_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/rows_ab.py --rows 1000000 --batch 1000000 --configs "nodes;rows@v1;rows" > gpurun_out/ab2_c2.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/rows_ab.py --rows 3700000000 --batch 8000000 --configs "rows@v1;rows;rows:128,4" > gpurun_out/ab2_c4.log 2>&1 || exit 1
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_BRANCH"
P2="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $P --kernel-include-regex k_traverse_rows -d gpurun_out/sq_$i -o run --output-format csv -- python tools/rows_ab.py --rows 400000000 --batch 8000000 --steps 3 --configs rows > gpurun_out/sq_$i.log 2>&1 || exit 1
done
