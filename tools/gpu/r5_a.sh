# r05 step A: where the C4 traversal's time goes -- per-phase shader-clock
# stamps (tools/_ab/libmbrwt_stamps.so), no-walk and cache-resident-block
# variants, SQ counters of the release k_traverse_rows
set -o pipefail
O=gpurun_out/r5a; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/trav_ab.py --tag release > $O/trav_release.log 2>&1 || exit 1
for v in stamps nowalk hot; do
MBRWT_LIB=tools/_ab/libmbrwt_$v.so timeout -k 10 300 python -u tools/trav_ab.py --tag $v > $O/trav_$v.log 2>&1 || exit 1
done
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH"
C="TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum GRBM_GUI_ACTIVE GRBM_COUNT SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_WR SQ_INSTS_SMEM"
i=0
for P in "$A" "$B" "$C"; do i=$((i+1))
timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex k_traverse_rows -d $O/sq$i -o run --output-format csv -- python tools/trav_ab.py --steps 3 --warmup 2 --tag sq$i > $O/sq$i.log 2>&1 || exit 1
done
timeout -k 10 120 python -u tools/pcie_probe.py > $O/pcie_probe.log 2>&1 || exit 1
