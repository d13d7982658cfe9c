# r05 step AB: non-temporal stores in the pageable host path's staging ->
# caller copies vs plain memcpy, same box, three rounds interleaved; the
# host-path GPU tests first
set -o pipefail
O=gpurun_out/r5ab; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hostpipe.py > $O/tests.log 2>&1 || exit 1
B="--steps 5 --warmup 2 --no-cpu --no-probe --traffic off"
for r in 1 2 3; do
timeout -k 10 300 python -u bench.py $B > $O/bench_nt_$r.log 2>&1 || exit 1
MBRWT_LIB=tools/_ab/libmbrwt_plaincopy.so timeout -k 10 300 python -u bench.py $B > $O/bench_plain_$r.log 2>&1 || exit 1
done
