set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log | grep -q "pytest rc=0" || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD" "SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_WAVES SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex k_traverse_fast2 -d gpurun_out/sq_c4_$i -o run --output-format csv -- python tools/sweep.py --variants 18 --reps 2 > gpurun_out/sq_c4_$i.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex k_traverse_fast2 -d gpurun_out/sq_c2_$i -o run --output-format csv -- python tools/sweep.py --rows 1000000 --variants 17 --reps 2 > gpurun_out/sq_c2_$i.log 2>&1 || exit 1
done
