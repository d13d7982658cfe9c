# r05 step AE: (1) the mad24 + linear-path change against neither, in ABBA
# order (the r5_z rounds always ran the release first); (2) what the spill
# reloads cost -- one row per 64-byte block (no spills, 237 GB) against two
set -o pipefail
O=gpurun_out/r5ae; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NO=tools/_ab/libmbrwt_noasm24.so
for r in 1 2; do
timeout -k 10 300 python -u tools/trav_ab.py --tag relA$r > $O/c4_relA_$r.log 2>&1 || exit 1
MBRWT_LIB=$NO timeout -k 10 300 python -u tools/trav_ab.py --tag noB$r > $O/c4_noB_$r.log 2>&1 || exit 1
MBRWT_LIB=$NO timeout -k 10 300 python -u tools/trav_ab.py --tag noC$r > $O/c4_noC_$r.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/trav_ab.py --tag relD$r > $O/c4_relD_$r.log 2>&1 || exit 1
done
timeout -k 10 400 python -u tools/trav_ab.py --rows-block 64,1 --tag s1 > $O/c4_s1.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/trav_ab.py --tag s2 > $O/c4_s2.log 2>&1 || exit 1
