set -o pipefail
mkdir -p gpurun_out/sq
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY"
for v in rows rows@diag1 rows@w5; do
  tag=$(echo $v | tr '@' '_')
  timeout -s KILL 240 rocprofv3 --pmc $C -d gpurun_out/sq/$tag -o run --output-format csv -- python tools/rows_ab.py --rows 3700000000 --batch 8000000 --steps 3 --configs "$v" > gpurun_out/sq/$tag.log 2>&1 || exit 1
done
