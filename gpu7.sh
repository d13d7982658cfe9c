set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/gather_probe 120 > gpurun_out/probe2.log 2>&1 || echo "probe rc=$?" >> gpurun_out/probe2.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_traverse_group -d gpurun_out/pmc_fetch -o run --output-format csv -- python tools/sweep.py --variants 3 --reps 1 > gpurun_out/pmc_fetch.log 2>&1; echo "rc=$?" >> gpurun_out/pmc_fetch.log
timeout -k 10 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex k_traverse_group -d gpurun_out/pmc_hit -o run --output-format csv -- python tools/sweep.py --variants 3 --reps 1 > gpurun_out/pmc_hit.log 2>&1; echo "rc=$?" >> gpurun_out/pmc_hit.log
timeout -k 10 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-include-regex k_traverse_group -d gpurun_out/pmc_rdreq -o run --output-format csv -- python tools/sweep.py --variants 3 --reps 1 > gpurun_out/pmc_rdreq.log 2>&1; echo "rc=$?" >> gpurun_out/pmc_rdreq.log
