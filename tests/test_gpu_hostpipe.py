"""The host-buffer get_rows (include/mbrwt.h mbrwt_get_rows; csrc/hostpipe.cpp):
host row ids -> host CSR, cut into chunks of 2^20 rows whose upload, query
and download overlap.  Checked against the oracle over batches of several
chunks, with pageable (numpy) and page-locked (torch pin_memory) buffers,
the capacity protocol, a row out of range in a later chunk, and chunks
denser than the slot estimate (the re-run path)."""
import ctypes as C

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def _ptr(a, t):
    import torch
    addr = a.data_ptr() if isinstance(a, torch.Tensor) else a.ctypes.data
    return C.cast(C.c_void_p(addr), C.POINTER(t))


def _call(dev, rows, offsets, cols, cap):
    from genome_graph_annotation_amd import _lib as L
    need = C.c_uint64(0)
    st = L.lib().mbrwt_get_rows(dev._h, _ptr(rows, C.c_uint64), len(rows), _ptr(offsets, C.c_uint64),
                                _ptr(cols, C.c_uint32) if cols is not None else None, cap, C.byref(need))
    return st, int(need.value)


@pytest.fixture(scope="module")
def c2(oracle_mod):
    from genome_graph_annotation_amd import BRWTDevice
    n, m, d = 1_000_000, 2652, 0.003
    return BRWTDevice.synthetic(n, m, d, 8, 42), oracle_mod.OracleTree.topdown(n, m, d, 8, 42), n


@pytest.mark.parametrize("pinned", ["none", "all", "rows", "outputs"])
def test_host_pipeline_chunks(c2, pinned):
    import torch
    from genome_graph_annotation_amd import _lib as L
    dev, ref, n = c2
    q = np.random.default_rng(5).integers(0, n, 2 * (1 << 20) + 12_345, dtype=np.uint64)
    off_o, cols_o = ref.get_rows(q)
    tot = len(cols_o)
    rows = torch.from_numpy(q.view(np.int64)).pin_memory() if pinned in ("all", "rows") else q
    if pinned in ("all", "outputs"):
        offsets = torch.zeros(len(q) + 1, dtype=torch.int64).pin_memory()
        cols = torch.zeros(tot + 7, dtype=torch.int32).pin_memory()
    else:
        offsets = np.zeros(len(q) + 1, dtype=np.uint64)
        cols = np.zeros(tot + 7, dtype=np.uint32)
    st, need = _call(dev, rows, offsets, cols, tot + 7)
    assert st == L.MBRWT_OK and need == tot
    o = offsets.numpy().view(np.uint64) if isinstance(offsets, torch.Tensor) else offsets
    c = cols.numpy().view(np.uint32) if isinstance(cols, torch.Tensor) else cols
    np.testing.assert_array_equal(o, off_o)
    np.testing.assert_array_equal(c[:tot], cols_o)


def test_host_pipeline_capacity_and_range(c2):
    from genome_graph_annotation_amd import _lib as L
    dev, ref, n = c2
    q = np.random.default_rng(6).integers(0, n, (1 << 20) + 999, dtype=np.uint64)
    off_o, cols_o = ref.get_rows(q)
    tot = len(cols_o)
    offsets = np.zeros(len(q) + 1, dtype=np.uint64)
    # count only, then one label short, then exact
    st, need = _call(dev, q, offsets, None, 0)
    assert st == L.MBRWT_ERR_CAPACITY and need == tot
    cols = np.zeros(tot, dtype=np.uint32)
    st, need = _call(dev, q, offsets, cols, tot - 1)
    assert st == L.MBRWT_ERR_CAPACITY and need == tot
    st, need = _call(dev, q, offsets, cols, tot)
    assert st == L.MBRWT_OK and need == tot
    np.testing.assert_array_equal(offsets, off_o)
    np.testing.assert_array_equal(cols, cols_o)
    # a row out of range in the second chunk
    bad = q.copy()
    bad[(1 << 20) + 5] = n
    st, _ = _call(dev, bad, offsets, cols, tot + 100)
    assert st == L.MBRWT_ERR_RANGE
    # the context still answers afterwards; an empty batch
    off_d, cols_d = dev.get_rows(q[:1000])
    np.testing.assert_array_equal(cols_d, cols_o[:off_o[1000]])
    off_e, cols_e = dev.get_rows(np.zeros(0, dtype=np.uint64))
    assert off_e.tolist() == [0] and len(cols_e) == 0


def test_host_pipeline_dense_chunks(oracle_mod):
    """Chunks far denser than the matrix's mean row: the slot's label estimate
    overflows and the chunk is queried again with room."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    n, m = 20_000, 64
    dense = np.zeros((n, m), dtype=bool)
    dense[:100] = True
    t = O.OracleTree.from_dense(dense, "basic", 8)
    dev = BRWTDevice.from_tree(t.export())
    q = np.random.default_rng(7).integers(0, 100, (1 << 20) + 50_000, dtype=np.uint64)
    off_o, cols_o = t.get_rows(q)
    off_d, cols_d = dev.get_rows(q)
    np.testing.assert_array_equal(off_d, off_o)
    np.testing.assert_array_equal(cols_d, cols_o)


@pytest.mark.parametrize("fail_at", [1, 3])
def test_host_pipeline_error_drains_inflight_copies(c2, fail_at):
    """An error return in the middle of a batch (an injected NOMEM when chunk
    `fail_at` is issued, MBRWT_OPT_TEST_FAIL_CHUNK) comes back only after the
    chunks already queued have finished: nothing lands in the caller's
    page-locked buffers after the call returned, and the context
    answers correctly afterwards."""
    import time
    import torch
    from genome_graph_annotation_amd import _lib as L
    dev, ref, n = c2
    q = np.random.default_rng(9).integers(0, n, 5 * (1 << 20) + 77, dtype=np.uint64)
    rows = torch.from_numpy(q.view(np.int64)).pin_memory()
    offsets = torch.zeros(len(q) + 1, dtype=torch.int64).pin_memory()
    cols = torch.zeros(len(q) * 12, dtype=torch.int32).pin_memory()
    dev.set_option(L.MBRWT_OPT_TEST_FAIL_CHUNK, fail_at)
    try:
        st, _ = _call(dev, rows, offsets, cols, cols.numel())
    finally:
        dev.set_option(L.MBRWT_OPT_TEST_FAIL_CHUNK, -1)
    assert st == L.MBRWT_ERR_NOMEM
    snap_o, snap_c = offsets.clone(), cols.clone()
    time.sleep(0.3)  # (a DMA still running would change the buffers now)
    assert torch.equal(offsets, snap_o) and torch.equal(cols, snap_c)
    off_o, cols_o = ref.get_rows(q[:300_000])
    off_d, cols_d = dev.get_rows(q[:300_000])
    np.testing.assert_array_equal(off_d, off_o)
    np.testing.assert_array_equal(cols_d, cols_o)
