set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS --kernel-include-regex k_traverse_group -d gpurun_out/pmc_sq -o run --output-format csv -- python tools/sweep.py --variants 3 --reps 1 > gpurun_out/pmc_sq.log 2>&1; echo "rc=$?" >> gpurun_out/pmc_sq.log
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-include-regex k_traverse_group -d gpurun_out/pmc_tcc -o run --output-format csv -- python tools/sweep.py --variants 3 --reps 1 > gpurun_out/pmc_tcc.log 2>&1; echo "rc=$?" >> gpurun_out/pmc_tcc.log
