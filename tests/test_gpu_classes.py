"""GPU parity of RECORD CLASSES (csrc/rows_class.hip, include/mbrwt.h
MBRWT_BUILD_ROWS_CLASSES): row-record images that keep one copy of every
distinct record plus a per-row class index, against the CPU oracle on the
reference's own correlated generator (`uniform_rows`,
experiments/main.cpp:232-247, data_generation.cpp:114-139, restated in
oracle/brwt_oracle.cpp) -- bit-exact get_rows (host, device, asynchronous),
point queries, columns, count_labels, the V / L accounting, errors, export
and serialization -- and the AUTO policy (classes on repeated rows, none on
i.i.d. columns).
"""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def _classes_build(value, fn):
    from genome_graph_annotation_amd import _lib as L
    from genome_graph_annotation_amd.brwt import build_option
    with build_option(L.MBRWT_BUILD_ROWS_CLASSES, value):
        return fn()


def _uniform_rows(O, n, m, d, unique, part, arity, relax):
    words, nr = O.generate_uniform_rows(n, m, d, unique, 42)
    return O.OracleTree.from_words(words, nr, m, part, arity, relax), nr


def _check(O, t, dev, rows):
    from test_gpu_rows import _check_all, _count_labels
    off_o, cols_o, vis = t.get_rows(rows, with_visits=True)
    _check_all(t, dev, rows)
    m = t.num_columns()
    want = np.bincount(cols_o.astype(np.int64), minlength=m).astype(np.uint64)
    np.testing.assert_array_equal(_count_labels(dev, rows), want)
    import torch
    rt = torch.from_numpy(np.ascontiguousarray(rows).view(np.int64)).cuda()
    assert dev.count_work_device(rt) == (int(vis.sum()), len(cols_o))


@pytest.mark.parametrize("part,arity,relax", [("basic", 8, 0), ("basic", 2, 0), ("greedy", 2, 10)])
@pytest.mark.parametrize("mode", [1, -1])
def test_classes_uniform_rows(oracle_mod, part, arity, relax, mode):
    """uniform_rows (500 distinct rows x 400): every query on the classes."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    t, n = _uniform_rows(O, 200_000, 300, 0.01, 500, part, arity, relax)
    dev = _classes_build(mode, lambda: BRWTDevice.from_tree(t.export(), layout="rows"))
    st = dev.rows_stats()
    assert 0 < st["classes"] <= 500 and st["rows_per_block"] == 1
    assert (1 << st["class_bits"]) >= st["classes"] > (1 << (st["class_bits"] - 1))
    plain = _classes_build(0, lambda: BRWTDevice.from_tree(t.export(), layout="rows"))
    assert plain.rows_stats()["classes"] == 0
    assert 2 * dev.device_bytes() <= plain.device_bytes()
    rng = np.random.default_rng(5)
    rows = np.concatenate([np.arange(0, n, 97), rng.integers(0, n, 60_000), [n - 1]]).astype(np.uint64)
    _check(O, t, dev, rows)


def test_classes_iid_auto_declines_forced_exact(oracle_mod):
    """i.i.d. columns: AUTO builds no classes (almost every record distinct);
    forced classes hold one class per distinct record and stay exact."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    rng = np.random.default_rng(9)
    n, m = 30_000, 120
    dense = rng.random((n, m)) < 0.04
    dense[:500] = False  # a class of empty rows
    t = O.OracleTree.from_dense(dense, "basic", 4)
    auto = _classes_build(-1, lambda: BRWTDevice.from_tree(t.export(), layout="rows"))
    assert auto.rows_stats()["classes"] == 0
    forced = _classes_build(1, lambda: BRWTDevice.from_tree(t.export(), layout="rows"))
    distinct = len({r.tobytes() for r in np.packbits(dense, axis=1)})
    assert forced.rows_stats()["classes"] == distinct
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 20_000)]).astype(np.uint64)
    _check(O, t, forced, rows)


def test_classes_sampled_auto(oracle_mod):
    """Beyond 2^20 rows AUTO decides on a strided sample first."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    t, n = _uniform_rows(O, 1_500_000, 200, 0.02, 3000, "basic", 8, 0)
    dev = _classes_build(-1, lambda: BRWTDevice.from_tree(t.export(), layout="rows"))
    st = dev.rows_stats()
    assert 0 < st["classes"] <= 3000 and 0 < st["class_sample_distinct"] <= 3000
    rows = np.random.default_rng(2).integers(0, n, 200_000).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    off_d, cols_d = dev.get_rows(rows)
    np.testing.assert_array_equal(off_d, off_o)
    np.testing.assert_array_equal(cols_d, cols_o)


def test_classes_errors_async_export(oracle_mod):
    """Range errors (host and asynchronous), the asynchronous call, and the
    export / serialization of a classes image (the same bytes as the node
    image's serialization of the same tree)."""
    O = oracle_mod
    import torch
    from genome_graph_annotation_amd import BRWTDevice, MBRWTError, _lib as L
    t, n = _uniform_rows(O, 50_000, 150, 0.03, 200, "basic", 4, 0)
    dev = _classes_build(1, lambda: BRWTDevice.from_tree(t.export(), layout="rows"))
    assert dev.rows_stats()["classes"] > 0
    with pytest.raises(MBRWTError) as ei:
        dev.get_rows(np.array([0, n], dtype=np.uint64))
    assert ei.value.status == L.MBRWT_ERR_RANGE
    with pytest.raises(MBRWTError):
        dev.get_batch([n], [0])
    s = torch.cuda.current_stream().cuda_stream
    st = torch.zeros(3, dtype=torch.int64, device="cuda")
    rng = np.random.default_rng(4)
    outs = []
    for k in (1, 64, 65, 9000):
        rows = rng.integers(0, n, k).astype(np.uint64)
        rt = torch.from_numpy(rows.view(np.int64)).cuda()
        ot = torch.empty(k + 1, dtype=torch.int64, device="cuda")
        ct = torch.empty(k * 40 + 64, dtype=torch.int32, device="cuda")
        dev.get_rows_device_async(rt, ot, ct, st, s)
        outs.append((rows, ot, ct, st.clone()))
    torch.cuda.synchronize()
    for rows, ot, ct, st_k in outs:
        off_o, cols_o = t.get_rows(rows)
        need, status, _ = st_k.cpu().tolist()
        assert status == L.MBRWT_OK and need == len(cols_o)
        np.testing.assert_array_equal(ot.cpu().numpy().view(np.uint64), off_o)
        np.testing.assert_array_equal(ct[:need].cpu().numpy().view(np.uint32), cols_o)
    bad = torch.tensor([0, n], dtype=torch.int64, device="cuda")
    st.zero_()
    dev.get_rows_device_async(bad, torch.empty(3, dtype=torch.int64, device="cuda"),
                              torch.empty(1000, dtype=torch.int32, device="cuda"), st, s)
    torch.cuda.synchronize()
    assert st.cpu().tolist()[1] == L.MBRWT_ERR_RANGE
    nodes = BRWTDevice.from_tree(t.export(), layout="nodes")
    assert dev.serialize() == nodes.serialize()
    back = BRWTDevice.load(dev.serialize(), layout="nodes")
    rows = rng.integers(0, n, 5000).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    off_b, cols_b = back.get_rows(rows)
    np.testing.assert_array_equal(off_b, off_o)
    np.testing.assert_array_equal(cols_b, cols_o)
