# r05 step G: the next tile's blocks requested while this tile is walked
# (register prefetch, spill loads first), persistent and 4-tile grids
set -o pipefail
O=gpurun_out/r5g; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/trav_ab.py --tag release > $O/trav_release.log 2>&1 || exit 1
for v in pf tpw1 pf_tpw4 pf_stamps; do
MBRWT_LIB=tools/_ab/libmbrwt_$v.so timeout -k 10 300 python -u tools/trav_ab.py --tag $v --stamps-out $O/stamps_$v.npy > $O/trav_$v.log 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dist.py tests/test_gpu_wire.py tests/test_gpu_rows.py tests/test_gpu_shards.py > $O/tests_dist.log 2>&1 || exit 1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --dist-backend gloo --rows 1000000000 --steps 10 --warmup 3 --no-e2e > $O/rehearsal_2rank.log 2>&1 || exit 1
