set -o pipefail
mkdir -p gpurun_out/fp gpurun_out/sq3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"
timeout -s KILL 240 rocprofv3 --pmc $C -d gpurun_out/sq3/a -o run --output-format csv -- python tools/rows_ab.py --rows 3700000000 --batch 8000000 --steps 3 --configs "rows" > gpurun_out/sq3/a.log 2>&1 || exit 1
C2="TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_ANY"
timeout -s KILL 240 rocprofv3 --pmc $C2 -d gpurun_out/sq3/b -o run --output-format csv -- python tools/rows_ab.py --rows 3700000000 --batch 8000000 --steps 3 --configs "rows" > gpurun_out/sq3/b.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/bench_wire.py > gpurun_out/fp/bench_wire.log 2>&1 || exit 1
timeout -k 10 700 python -u tools/footprint.py > gpurun_out/fp/footprint.log 2>&1 || exit 1
