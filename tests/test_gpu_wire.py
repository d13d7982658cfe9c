"""GPU parity of the device-sized all-gatherv wire (include/mbrwt.h
mbrwt_pack_csr_device / mbrwt_unpack_labels_device; dist.DeviceAllGatherV):
per-rank CSR slices computed on the device with the asynchronous get_rows
(label counts only on the device), packed into fixed-size wire segments, the
segments concatenated as an all-gather would, and unpacked into the global
CSR -- against the oracle's CSR of the whole batch.  Covers several segments,
an empty slice, 12- and 32-bit wires and the capacity-overflow flag; and the
DeviceAllGatherV class itself over a one-rank RCCL group."""
import ctypes as C

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def _slices(O, n_batch, world, num_columns, seed=5):
    import torch
    from genome_graph_annotation_amd import BRWTDevice
    from genome_graph_annotation_amd.dist import shard_bounds
    n = 60_000
    t = O.OracleTree.topdown(n, 2652, 0.003, 8, 11)
    dev = BRWTDevice.from_tree(t.export(), layout="rows")
    rows = np.random.default_rng(seed).integers(0, n, n_batch, dtype=np.uint64)
    out = []
    for r in range(world):
        lo, hi = shard_bounds(n_batch, world, r)
        rt = torch.from_numpy(np.ascontiguousarray(rows[lo:hi]).view(np.int64)).cuda()
        off = torch.zeros(hi - lo + 1, dtype=torch.int64, device="cuda")
        cols = torch.zeros(20 * (hi - lo) + 64, dtype=torch.int32, device="cuda")
        st = torch.zeros(3, dtype=torch.int64, device="cuda")
        if hi > lo:
            dev.get_rows_device_async(rt, off, cols, st, torch.cuda.current_stream().cuda_stream)
        out.append((hi - lo, off, cols, st))
    torch.cuda.synchronize()
    return t, rows, out


@pytest.mark.parametrize("world,n_batch,num_columns", [(3, 30_001, 2652), (4, 3, 2652), (2, 10_000, None),
                                                     (8, 40_003, 2652), (5, 20_001, 5000)])
def test_wire_segments_reassemble(oracle_mod, world, n_batch, num_columns):
    import torch
    from genome_graph_annotation_amd import _lib as L
    from genome_graph_annotation_amd.dist import _round16, _words, wire_bits
    t, rows, sl = _slices(oracle_mod, n_batch, world, num_columns)
    bits_l, bits_c = wire_bits(num_columns)
    ns = [x[0] for x in sl]
    cap = max(int(x[3][0].item()) for x in sl) + 5
    lab_off = int(L.lib().mbrwt_wire_labels_offset(max(ns), bits_c))
    per = _round16(lab_off + max(1, (cap + 31) // 32 * bits_l) * 4)
    recv = torch.full((world * per,), 0xAB, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for r, (nr, off, cols, st) in enumerate(sl):
        seg = recv[r * per:(r + 1) * per]
        L.check(L.lib().mbrwt_pack_csr_device(off.data_ptr(), nr, cols.data_ptr(), cols.numel(), st.data_ptr(), cap, bits_c,
                                              bits_l, lab_off, seg.data_ptr(), per, s), "pack")
    N = sum(ns)
    cnt = torch.zeros(max(1, N), dtype=torch.int32, device="cuda")
    g_cols = torch.zeros(world * cap + 32, dtype=torch.int32, device="cuda")
    status = torch.full((2,), -1, dtype=torch.int64, device="cuda")
    arr = (C.c_uint64 * world)(*ns)
    L.check(L.lib().mbrwt_unpack_segments_device(recv.data_ptr() + 8, world, per, arr, bits_c, cnt.data_ptr(), s),
            "unpack counts")
    L.check(L.lib().mbrwt_unpack_labels_device(recv.data_ptr(), world, per, lab_off, cap, bits_l,
                                               g_cols.data_ptr(), g_cols.numel(), status.data_ptr(), s),
            "unpack labels")
    torch.cuda.synchronize()
    off_o, cols_o = t.get_rows(rows)
    tot, bad = status.tolist()
    assert bad == 0 and tot == len(cols_o)
    g_off = np.concatenate([[0], np.cumsum(cnt[:N].cpu().numpy().astype(np.uint64))]).astype(np.uint64)
    np.testing.assert_array_equal(g_off, off_o)
    np.testing.assert_array_equal(g_cols[:tot].cpu().numpy().view(np.uint32), cols_o)
    # the global offsets straight from the packed counts (r04: three-pass scan)
    tb = C.c_uint64(0)
    L.check(L.lib().mbrwt_unpack_offsets_device(recv.data_ptr(), world, per, arr, bits_c, None, None, C.byref(tb), s),
            "offsets scratch")
    tmp = torch.zeros(max(16, int(tb.value)), dtype=torch.uint8, device="cuda")
    off_d = torch.full((N + 1,), -1, dtype=torch.int64, device="cuda")
    L.check(L.lib().mbrwt_unpack_offsets_device(recv.data_ptr(), world, per, arr, bits_c, off_d.data_ptr(),
                                                tmp.data_ptr(), C.byref(tb), s), "offsets")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(off_d.cpu().numpy().view(np.uint64), off_o)
    if world <= 8:  # (nine segments: beyond one node, the call declines)
        arr9 = (C.c_uint64 * 9)(*([1] * 9))
        assert L.lib().mbrwt_unpack_offsets_device(recv.data_ptr(), 9, per, arr9, bits_c, None, None,
                                                   C.byref(tb), s) == L.MBRWT_ERR_UNSUPPORTED
    # a label capacity below a slice's count: flagged, nothing written
    small = min(int(x[3][0].item()) for x in sl if x[0] > 0)
    if small > 1:
        cap2 = small - 1
        per2 = _round16(lab_off + max(1, (cap2 + 31) // 32 * bits_l) * 4)
        recv2 = torch.zeros(world * per2, dtype=torch.uint8, device="cuda")
        for r, (nr, off, cols, st) in enumerate(sl):
            seg = recv2[r * per2:(r + 1) * per2]
            L.check(L.lib().mbrwt_pack_csr_device(off.data_ptr(), nr, cols.data_ptr(), cols.numel(), st.data_ptr(), cap2, bits_c,
                                                  bits_l, lab_off, seg.data_ptr(), per2, s), "pack")
        g2 = torch.full((world * cap2 + 32,), 7, dtype=torch.int32, device="cuda")
        L.check(L.lib().mbrwt_unpack_labels_device(recv2.data_ptr(), world, per2, lab_off, cap2, bits_l,
                                                   g2.data_ptr(), g2.numel(), status.data_ptr(), s), "unpack")
        torch.cuda.synchronize()
        assert status[1].item() == 1
        assert bool((g2 == 7).all())
    # a rank whose own CSR is smaller than its label count (its get_rows
    # failed on capacity): flagged through the header, its CSR never read
    big = max(range(world), key=lambda r: int(sl[r][3][0].item()))
    nb = int(sl[big][3][0].item())
    if nb > 1:
        recv3 = torch.zeros(world * per, dtype=torch.uint8, device="cuda")
        for r, (nr, off, cols, st) in enumerate(sl):
            seg = recv3[r * per:(r + 1) * per]
            ccap = nb - 1 if r == big else cols.numel()
            L.check(L.lib().mbrwt_pack_csr_device(off.data_ptr(), nr, cols.data_ptr(), ccap, st.data_ptr(), cap,
                                                  bits_c, bits_l, lab_off, seg.data_ptr(), per, s), "pack")
        g3 = torch.full((world * cap + 32,), 7, dtype=torch.int32, device="cuda")
        status.fill_(-1)
        L.check(L.lib().mbrwt_unpack_labels_device(recv3.data_ptr(), world, per, lab_off, cap, bits_l,
                                                   g3.data_ptr(), g3.numel(), status.data_ptr(), s), "unpack")
        torch.cuda.synchronize()
        assert status[1].item() == 1
        assert bool((g3 == 7).all())


def test_device_allgatherv_one_rank(oracle_mod):
    """DeviceAllGatherV (bench.py's N > 1 exchange) over a one-rank RCCL group:
    pipelined start / finish on two slots, every result against the oracle."""
    import torch
    import torch.distributed as dist
    from genome_graph_annotation_amd import BRWTDevice
    from genome_graph_annotation_amd.dist import DeviceAllGatherV
    O = oracle_mod
    store = dist.HashStore()
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        n = 50_000
        t = O.OracleTree.topdown(n, 2652, 0.003, 8, 12)
        dev = BRWTDevice.from_tree(t.export(), layout="rows")
        batches = [np.random.default_rng(70 + k).integers(0, n, 20_000, dtype=np.uint64) for k in range(3)]
        wire = DeviceAllGatherV([20_000], 20_000 * 12, 2652, torch.device("cuda", 0), timing=True)
        s = torch.cuda.current_stream().cuda_stream
        st = torch.zeros(3, dtype=torch.int64, device="cuda")
        bufs = [(torch.zeros(20_001, dtype=torch.int64, device="cuda"),
                 torch.zeros(20_000 * 12, dtype=torch.int32, device="cuda")) for _ in range(2)]
        pending, results = None, []
        for k, b in enumerate(batches):
            o, cb = bufs[k % 2]
            dev.get_rows_device_async(torch.from_numpy(b.view(np.int64)).cuda(), o, cb, st, s)
            if pending is not None:
                g = wire.finish(pending)
                results.append(tuple(x.clone() for x in g))
            pending = wire.start(o, cb, st)
        g = wire.finish(pending)
        results.append(tuple(x.clone() for x in g))
        torch.cuda.synchronize()
        for b, (g_off, g_cols, g_st) in zip(batches, results):
            off_o, cols_o = t.get_rows(b)
            tot, bad = g_st.tolist()
            assert bad == 0 and tot == len(cols_o)
            np.testing.assert_array_equal(g_off.cpu().numpy().view(np.uint64), off_o)
            np.testing.assert_array_equal(g_cols[:tot].cpu().numpy().view(np.uint32), cols_o)
        ph = wire.phases()
        assert set(ph) == {"pack_ms", "all_gather_ms", "unpack_ms"}
    finally:
        dist.destroy_process_group()
