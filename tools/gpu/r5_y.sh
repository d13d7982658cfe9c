# r05 step Y: copy threads of the pageable host path (15 vs the r05 7), same
# box, two rounds interleaved (bench.py's end_to_end leg)
set -o pipefail
O=gpurun_out/r5y; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="--steps 5 --warmup 2 --no-cpu --no-probe --traffic off"
for r in 1 2; do
timeout -k 10 300 python -u bench.py $B > $O/bench_pool15_$r.log 2>&1 || exit 1
MBRWT_LIB=tools/_ab/libmbrwt_pool7.so timeout -k 10 300 python -u bench.py $B > $O/bench_pool7_$r.log 2>&1 || exit 1
done
