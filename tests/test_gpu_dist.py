"""The N > 1 step of bench.py on a real GPU, two ranks on GPU 0: every rank
traverses its contiguous slice of each global batch with the asynchronous
get_rows (row records, the library default), and dist.DeviceAllGatherV
reassembles the global CSR pipelined over 3 wire slots (up to two exchanges
in flight behind the current step, no host synchronisation per step), the
batches alternating between two query contexts on two streams -- the exact
call pattern of bench.py at N > 1.  The process group is gloo (two
processes sharing one GPU cannot form an RCCL group); on the 8-GPU node the
same code runs over RCCL.  Every reassembled batch is checked against the
oracle."""
import os
import socket
import sys

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as O
        from genome_graph_annotation_amd import BRWTDevice
        from genome_graph_annotation_amd.dist import DeviceAllGatherV, shard_bounds
        torch.cuda.set_device(0)
        dev_t = torch.device("cuda", 0)
        n, m, d, G, K = 400_000, 2652, 0.003, 100_001, 6
        mat = BRWTDevice.synthetic(n, m, d, 8, 31)
        assert mat.layout() == "rows"
        lo, hi = shard_bounds(G, world, rank)
        nb = hi - lo
        globals_np = [np.random.default_rng(500 + k).integers(0, n, G, dtype=np.uint64) for k in range(K)]
        rows_ts = [torch.from_numpy(np.ascontiguousarray(g[lo:hi]).view(np.int64)).to(dev_t) for g in globals_np]
        # each rank sizes its own capacity from its own slice (they differ:
        # r4c's gloo abort); DeviceAllGatherV agrees on the largest itself
        cap = int(nb * 8 * 1.3) + 1024 + 24 * rank
        rows_per_rank = [shard_bounds(G, world, r)[1] - shard_bounds(G, world, r)[0] for r in range(world)]
        wire = DeviceAllGatherV(rows_per_rank, cap, m, dev_t, slots=3)
        assert wire.cap == max(int(rows_per_rank[r] * 8 * 1.3) + 1024 + 24 * r for r in range(world))
        bufs = [(torch.empty(nb + 1, dtype=torch.int64, device=dev_t), torch.empty(cap, dtype=torch.int32, device=dev_t))
                for _ in range(2)]
        # bench.py's N > 1 step since r05: two query contexts (the context and
        # a clone over the same image) on two streams, alternating batches
        mats = [mat, mat.clone()]
        streams = [torch.cuda.current_stream(dev_t), torch.cuda.Stream(dev_t)]
        status = [torch.zeros(3, dtype=torch.int64, device=dev_t) for _ in range(2)]
        inflight, done = [], []
        for i in range(K):
            o, cb = bufs[i % 2]
            qi = i % 2
            with torch.cuda.stream(streams[qi]):
                mats[qi].get_rows_device_async(rows_ts[i], o, cb, status[qi], streams[qi].cuda_stream)
                if len(inflight) == len(wire.slots) - 1:
                    k, sl = inflight.pop(0)
                    g_off, g_cols, g_st = wire.finish(sl)
                    done.append((k, g_off.clone(), g_cols.clone(), g_st.clone()))
                inflight.append((i, wire.start(o, cb, status[qi])))
        while inflight:
            k, sl = inflight.pop(0)
            g_off, g_cols, g_st = wire.finish(sl)
            done.append((k, g_off.clone(), g_cols.clone(), g_st.clone()))
        torch.cuda.synchronize()
        # every asynchronous get_rows on both contexts returned MBRWT_OK
        ok = all(st.cpu().tolist()[2] == 1 for st in status)
        t = O.OracleTree.topdown(n, m, d, 8, 31)
        for k, g_off, g_cols, g_st in done:
            tot, bad = g_st.cpu().tolist()
            off_o, cols_o = t.get_rows(globals_np[k])
            ok = ok and bad == 0 and tot == len(cols_o)
            ok = ok and np.array_equal(g_off.cpu().numpy().view(np.uint64), off_o)
            ok = ok and np.array_equal(g_cols[:tot].cpu().numpy().view(np.uint32), cols_o)
        q.put((rank, bool(ok), len(done)))
    finally:
        dist.destroy_process_group()


def test_two_ranks_device_wire_pipelined(oracle_mod):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    res = sorted(q.get(timeout=5) for _ in range(world))
    assert [r[0] for r in res] == list(range(world))
    assert all(r[1] for r in res), res
    assert all(r[2] == 6 for r in res), res
    assert all(p.exitcode == 0 for p in procs)
