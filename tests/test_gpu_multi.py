"""GPU parity of the one-process multi-device path (include/mbrwt.h
"multi-device", csrc/multi.hip): replicas on devices [0] and [0, 0] (two
contexts on one device: the slices and the reassembly are the same code as
on N devices; peer copies become device-local copies), host and device
output buffers, node and row-record layouts, against the CPU oracle."""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


@pytest.mark.parametrize("devices", [(0,), (0, 0), (0, 0, 0)])
@pytest.mark.parametrize("layout", ["nodes", "rows"])
def test_multi_get_rows_like_oracle(oracle_mod, devices, layout):
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTMulti
    rng = np.random.default_rng(len(devices))
    n, m = 20000, 300
    dense = rng.random((n, m)) < 0.02
    t = O.OracleTree.from_dense(dense, "basic", 8)
    mu = BRWTMulti.from_tree(t.export(), devices=devices, layout=layout)
    assert mu.size() == len(devices)
    assert mu.replica(0).layout() == layout
    for k in (0, 1, 2, 7, 12345):  # batches shorter than, equal to and longer than the replica count
        rows = rng.integers(0, n, k).astype(np.uint64)
        off_o, cols_o = t.get_rows(rows)
        off_d, cols_d = mu.get_rows(rows)
        np.testing.assert_array_equal(off_d, off_o)
        np.testing.assert_array_equal(cols_d, cols_o)
    # device buffers on devices[0] (peer copies)
    import torch
    rows = rng.integers(0, n, 50000).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    rt = torch.from_numpy(rows.view(np.int64)).cuda()
    ot = torch.empty(len(rows) + 1, dtype=torch.int64, device="cuda")
    ct = torch.empty(len(cols_o) + 7, dtype=torch.int32, device="cuda")
    got = mu.get_rows_device(rt, ot, ct, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert got == len(cols_o)
    np.testing.assert_array_equal(ot.cpu().numpy().view(np.uint64), off_o)
    np.testing.assert_array_equal(ct[:got].cpu().numpy().view(np.uint32), cols_o)
    # capacity protocol
    from genome_graph_annotation_amd import _lib as L
    small = torch.empty(3, dtype=torch.int32, device="cuda")
    with pytest.raises(L.MBRWTError) as ei:
        mu.get_rows_device(rt, ot, small, torch.cuda.current_stream().cuda_stream)
    assert ei.value.status == L.MBRWT_ERR_CAPACITY and ei.value.needed == len(cols_o)


def test_multi_synthetic_and_errors(oracle_mod):
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTMulti, MBRWTError, _lib as L
    n, m, d = 300_000, 2652, 0.003
    mu = BRWTMulti.synthetic(n, m, d, 8, 42, devices=(0, 0), layout="rows")
    t = O.OracleTree.topdown(n, m, d, 8, 42)
    rows = np.random.default_rng(5).integers(0, n, 100_000).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    off_d, cols_d = mu.get_rows(rows)
    np.testing.assert_array_equal(off_d, off_o)
    np.testing.assert_array_equal(cols_d, cols_o)
    with pytest.raises(MBRWTError) as ei:
        mu.get_rows(np.array([0, n], dtype=np.uint64))
    assert ei.value.status == L.MBRWT_ERR_RANGE
    with pytest.raises(MBRWTError):
        BRWTMulti.synthetic(n, m, d, 8, 42, devices=(0, 99))
    # the failed creation leaves no sticky HIP error behind: the next query of
    # an ordinary context in this thread still succeeds (r03 regression: a
    # hipSetDevice(99) in the cleanup made the next launch check fail)
    from genome_graph_annotation_amd import BRWTDevice
    one = BRWTDevice.from_tree(O.OracleTree.from_dense(np.eye(5, dtype=bool), "basic", 2).export())
    off1, cols1 = one.get_rows(np.arange(5, dtype=np.uint64))
    assert cols1.tolist() == [0, 1, 2, 3, 4]
