"""Multi-process (world_size 2, gloo on CPU) coverage of the N>1 path:
batch sharding + the all-gatherv reassembly of per-rank CSR slices
(genome_graph_annotation_amd/dist.py; on GPUs the same code runs over RCCL).
Each rank's slice is computed by the oracle here (no GPU in this container)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_batch, q, num_columns=None, m=300):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as O
        from genome_graph_annotation_amd.dist import allgatherv_csr, shard_bounds
        t = O.OracleTree.topdown(50_000, m, 0.01 if m < 1000 else 0.002, 8, 3)
        rows = np.random.default_rng(9).integers(0, 50_000, n_batch, dtype=np.uint64)
        lo, hi = shard_bounds(n_batch, world, rank)
        off, cols = t.get_rows(rows[lo:hi])
        g_off, g_cols = allgatherv_csr(torch.from_numpy(off.view(np.int64)),
                                       torch.from_numpy(cols.view(np.int32)),
                                       n_labels=None if rank else int(off[-1]), num_columns=num_columns)
        ref_off, ref_cols = t.get_rows(rows)
        ok = np.array_equal(g_off.numpy().view(np.uint64), ref_off) and \
            np.array_equal(g_cols.numpy().view(np.uint32), ref_cols)
        q.put((rank, ok, int(hi - lo)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_batch,num_columns,m", [
    (2, 10_001, None, 300),      # 32-bit wire
    (2, 10_001, 300, 300),       # 9-bit wire (labels < 300, counts <= 300)
    (3, 4_001, 40_000, 40_000),  # 16-bit wire
    (2, 1, 300, 300),
    (3, 7, None, 300),
    (3, 2, 300, 300),            # a rank with an empty slice
])
def test_allgatherv_reassembles_global_csr(world, n_batch, num_columns, m):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_batch, q, num_columns, m)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res)
    assert sum(k for _, _, k in res) == n_batch


def test_shard_bounds_cover_batch():
    from genome_graph_annotation_amd.dist import shard_bounds
    for n in (0, 1, 7, 8, 1000, 8_000_001):
        for w in (1, 2, 3, 8):
            spans = [shard_bounds(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def test_wire_bit_packing_roundtrip():
    """dist.py's CPU bit-packing (the format of mbrwt_pack_ids_device) round-trips
    at every width, values spanning word boundaries."""
    from genome_graph_annotation_amd.dist import _pack, _unpack, _words
    rng = np.random.default_rng(5)
    for bits in (1, 3, 7, 12, 16, 17, 31, 32):
        n = 1000
        v = rng.integers(0, 1 << bits, n, dtype=np.uint64).astype(np.uint32)
        words = torch.zeros(_words(n, bits) + 1, dtype=torch.int32)
        _pack(torch.from_numpy(v.view(np.int32)), n, bits, words)
        out = torch.empty(n, dtype=torch.int32)
        _unpack(words, n, bits, out)
        assert np.array_equal(out.numpy().view(np.uint32), v)


def _pipelined_worker(rank, world, port, q):
    """bench.py's pipelined step shape: batch k's AllGatherV is started, batch
    k+1 is computed into the other output buffer, then batch k's exchange is
    finished; every finished global CSR must equal the oracle's answer for
    its own batch."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as O
        from genome_graph_annotation_amd.dist import AllGatherV, shard_bounds
        t = O.OracleTree.topdown(40_000, 2652, 0.003, 8, 4)
        batches = [np.random.default_rng(100 + k).integers(0, 40_000, 5_003 + 97 * k, dtype=np.uint64)
                   for k in range(4)]
        bufs = [None, None]
        pending, results = None, []
        for k, b in enumerate(batches):
            lo, hi = shard_bounds(len(b), world, rank)
            off, cols = t.get_rows(b[lo:hi])
            bufs[k % 2] = (torch.from_numpy(off.view(np.int64)).clone(), torch.from_numpy(cols.view(np.int32)).clone())
            if pending is not None:
                results.append(pending.finish())
            pending = AllGatherV(*bufs[k % 2], n_labels=int(off[-1]), num_columns=2652)
        results.append(pending.finish())
        ok = True
        for b, (g_off, g_cols) in zip(batches, results):
            ref_off, ref_cols = t.get_rows(b)
            ok &= np.array_equal(g_off.numpy().view(np.uint64), ref_off) and \
                np.array_equal(g_cols.numpy().view(np.uint32), ref_cols)
        q.put((rank, bool(ok), len(results)))
    finally:
        dist.destroy_process_group()


def test_pipelined_allgatherv_start_finish():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipelined_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok and n == 4 for _, ok, n in res)


def _agree_worker(rank, world, port, q, mismatch):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from genome_graph_annotation_amd.dist import _agree_wire
        ns = [5, 4, 4][:world]
        if mismatch == "rows" and rank == 1:
            ns = [4, 5, 4][:world]
        if mismatch == "length" and rank == 0:
            ns = ns + [4]  # (one entry too many on one rank only)
        m = 2652 + (1 if mismatch == "cols" and rank == world - 1 else 0)
        try:
            cap = _agree_wire(ns, 1000 + 24 * rank, m, None, torch.device("cpu"))
            q.put((rank, "ok", cap))
        except ValueError as e:
            q.put((rank, "error", str(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mismatch", [(2, None), (3, None), (2, "rows"), (3, "cols"), (2, "length"),
                                           (3, "length")])
def test_device_wire_agrees_on_layout(world, mismatch):
    """DeviceAllGatherV's collective precondition (the r4c
    gloo abort): ranks that pass different label capacities agree on the
    largest; ranks that pass different slices or column counts all raise the
    same ValueError before any wire collective (the exchange itself with
    per-rank capacities: tests/test_gpu_dist.py)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_worker, args=(r, world, port, q, mismatch)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    res = sorted(q.get(timeout=5) for _ in range(world))
    assert [r[0] for r in res] == list(range(world))
    if mismatch is None:
        assert all(r[1] == "ok" and r[2] == 1000 + 24 * (world - 1) for r in res), res
    else:
        assert all(r[1] == "error" for r in res), res
        assert len({r[2] for r in res}) == 1, res  # the same message on every rank
        assert ("num_columns" if mismatch == "cols" else "rows_per_rank") in res[0][2]
    assert all(p.exitcode == 0 for p in procs)
