# r05 step AG: SQ / TA counters of the FINAL k_traverse_rows at C4 (one tile
# per wave, DPP scans, full-rate mads, linear path table), one pass per group
set -o pipefail
O=gpurun_out/r5ag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH"
C="GRBM_COUNT GRBM_GUI_ACTIVE TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_WR"
i=0
for P in "$A" "$B" "$C"; do i=$((i+1))
timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex k_traverse_rows -d $O/sq$i -o run --output-format csv -- python tools/trav_ab.py --steps 3 --warmup 2 --tag sq$i > $O/sq$i.log 2>&1 || exit 1
done
