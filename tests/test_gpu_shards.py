"""Rows >= 2^32 through row shards (csrc/shards.hip).

The reference's Row is uint64_t (common/binary_matrix.hpp:11).  A context
over more rows than one device image addresses holds row shards -- the BRWT
restricted to consecutive row ranges -- and routes every query.  Bit-exact
against the oracle:
  * small trees with MBRWT_SHARD_ROWS forcing shards of 1..2048 rows (the
    routing, slicing and reassembly on the reference's grids and random
    trees, every query of the boundary);
  * the synthetic law over shards (node keys shifted by the positions of the
    earlier shards) against the oracle's unsharded tree of the same law;
  * a 4.5 B-row synthetic tree (3 shards of 2^31 rows) against the streamed
    oracle (no host structure), rows either side of 2^31, 2^32 and n - 1.
"""
import os

import numpy as np
import pytest

from conftest import gpu_available

# the per-node images (the library default, AUTO, builds row records:
# tests/test_gpu_rows.py); a test passing layout= explicitly overrides it
pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU"),
              pytest.mark.usefixtures("nodes_layout")]


def _env(name, value, fn):
    """fn() under the build option that replaced the r04 switch `name`."""
    from conftest import with_build
    return with_build(name, value, fn)


def _same_tree(a, b):
    from test_brwt_files import _same_tree as same
    same(a, b)


def _sharded(R, fn):
    return _env("MBRWT_SHARD_ROWS", str(R), fn)


def _check_all(O, t, dev, rng, n, m):
    from genome_graph_annotation_amd import _lib as L
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 3 * n), [n - 1, 0, n - 1]]).astype(np.uint64)
    rng.shuffle(rows)
    off_o, cols_o = t.get_rows(rows)
    from conftest import kernel_variants
    for v in kernel_variants(dev, (0, 1, 5, 10)):
        dev.set_option(L.MBRWT_OPT_KERNEL, v)
        off_d, cols_d = dev.get_rows(rows)
        np.testing.assert_array_equal(off_d, off_o)
        np.testing.assert_array_equal(cols_d, cols_o)
    dev.set_option(L.MBRWT_OPT_KERNEL, 0)
    # point queries
    qr = rng.integers(0, n, 4000).astype(np.uint64)
    qc = rng.integers(0, m, 4000).astype(np.uint64)
    np.testing.assert_array_equal(dev.get_batch(qr, qc), [t.get(int(r), int(c)) for r, c in zip(qr, qc)])
    # columns: ascending rows over the whole matrix
    for j in sorted({0, m // 2, m - 1}):
        np.testing.assert_array_equal(dev.get_column(j), np.asarray(t.get_column(j), dtype=np.uint64))
    # the tree read back: the shards' columns concatenated
    _same_tree(t.export(), dev.export())


@pytest.mark.parametrize("n,R", [(200, 7), (5000, 701), (5000, 2048)])
@pytest.mark.parametrize("build", [("basic", 2, 0), ("basic", 8, 0), ("greedy", 2, 4), ("greedy", 2, 0)])
def test_shards_from_tree(oracle_mod, n, R, build):
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    part, arity, relax = build
    rng = np.random.default_rng(R + arity)
    m = 40
    dense = rng.random((n, m)) < 0.1
    t = O.OracleTree.from_dense(dense, part, arity, relax)
    dev = _sharded(R, lambda: BRWTDevice.from_tree(t.export()))
    assert dev.num_shards() == (n + R - 1) // R
    assert dev.num_rows() == n and dev.num_columns() == m and dev.num_relations() == int(dense.sum())
    _check_all(O, t, dev, rng, n, m)


@pytest.mark.parametrize("kind", ["zero", "one", "mixed"])
def test_shards_reference_grids(oracle_mod, kind):
    """test_BRWT.cpp:152-212's grids with shards of 3 rows."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    for n in (4, 7, 19):
        for m in (1, 2, 5, 19):
            i = np.arange(n)[:, None]
            j = np.arange(m)[None, :]
            dense = {"zero": np.zeros((n, m), bool), "one": np.ones((n, m), bool),
                     "mixed": ((i + 2 * j) % 2).astype(bool)}[kind]
            t = O.OracleTree.from_dense(dense, "basic", 2, 0)
            dev = _sharded(3, lambda: BRWTDevice.from_tree(t.export()))
            assert dev.num_shards() == (n + 2) // 3
            off, cols = dev.get_rows(np.arange(n, dtype=np.uint64))
            off_o, cols_o = t.get_rows(np.arange(n, dtype=np.uint64))
            np.testing.assert_array_equal(off, off_o)
            np.testing.assert_array_equal(cols, cols_o)
            ii, jj = np.meshgrid(np.arange(n), np.arange(m), indexing="ij")
            np.testing.assert_array_equal(dev.get_batch(ii.ravel(), jj.ravel()), dense.ravel())


def test_shards_errors_and_empty(oracle_mod):
    from genome_graph_annotation_amd import BRWTDevice, _lib as L
    O = oracle_mod
    dense = np.random.default_rng(3).random((500, 20)) < 0.2
    t = O.OracleTree.from_dense(dense, "basic", 2, 0)
    dev = _sharded(64, lambda: BRWTDevice.from_tree(t.export()))
    assert dev.num_shards() == 8
    one_row = _sharded(1, lambda: BRWTDevice.from_tree(O.OracleTree.from_dense(dense[:9], "basic", 2, 0).export()))
    assert one_row.num_shards() == 9
    off1, cols1 = one_row.get_rows(np.array([8, 0, 4, 4], dtype=np.uint64))
    off1o, cols1o = O.OracleTree.from_dense(dense[:9], "basic", 2, 0).get_rows(np.array([8, 0, 4, 4], dtype=np.uint64))
    np.testing.assert_array_equal(off1, off1o)
    np.testing.assert_array_equal(cols1, cols1o)
    off, cols = dev.get_rows(np.zeros(0, dtype=np.uint64))
    assert len(off) == 1 and off[0] == 0 and len(cols) == 0
    with pytest.raises(L.MBRWTError):
        dev.get_rows(np.array([3, 500], dtype=np.uint64))
    with pytest.raises(L.MBRWTError):
        dev.get_batch(np.array([500], dtype=np.uint64), np.array([0], dtype=np.uint64))
    # rows of one shard only, the others idle
    off, cols = dev.get_rows(np.arange(128, 192, dtype=np.uint64))
    off_o, cols_o = t.get_rows(np.arange(128, 192, dtype=np.uint64))
    np.testing.assert_array_equal(off, off_o)
    np.testing.assert_array_equal(cols, cols_o)


def test_shards_device_api_and_classify(oracle_mod):
    """Device-buffer get_rows, count_labels and batched classify on a sharded
    context equal the unsharded context's answers (themselves oracle-checked
    in test_gpu_parity.py)."""
    import torch
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    rng = np.random.default_rng(9)
    n, m = 20000, 64
    dense = rng.random((n, m)) < 0.05
    t = O.OracleTree.from_dense(dense, "basic", 4, 0)
    one = BRWTDevice.from_tree(t.export())
    sh = _sharded(3001, lambda: BRWTDevice.from_tree(t.export()))
    assert sh.num_shards() == 7 and one.num_shards() == 1
    rows = rng.integers(0, n, 50_000).astype(np.uint64)
    rt = torch.from_numpy(rows.view(np.int64)).to("cuda:0")
    off_o, cols_o = t.get_rows(rows)
    ot = torch.empty(len(rows) + 1, dtype=torch.int64, device="cuda:0")
    ct = torch.empty(len(cols_o) + 1, dtype=torch.int32, device="cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    assert sh.get_rows_device(rt, ot, ct, s) == len(cols_o)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(ot.cpu().numpy().view(np.uint64), off_o)
    np.testing.assert_array_equal(ct[: len(cols_o)].cpu().numpy().view(np.uint32), cols_o)
    c1 = torch.zeros(m, dtype=torch.int64, device="cuda:0")
    c2 = torch.zeros(m, dtype=torch.int64, device="cuda:0")
    one.count_labels_device(rt, c1, s)
    sh.count_labels_device(rt, c2, s)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(c2.cpu().numpy(), np.bincount(cols_o, minlength=m))
    np.testing.assert_array_equal(c1.cpu().numpy(), c2.cpu().numpy())
    read_off = np.arange(0, len(rows) + 1, 50, dtype=np.uint64)
    for ratio in (0.0, 0.3, 1.0):
        a = one.get_labels_batch(rows, read_off, ratio)
        b = sh.get_labels_batch(rows, read_off, ratio)
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])
    a = one.get_top_labels_batch(rows, read_off, 5)
    b = sh.get_top_labels_batch(rows, read_off, 5)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    v1 = one.count_work_device(rt)
    v2 = sh.count_work_device(rt)
    assert v1[1] == v2[1] == len(cols_o)


@pytest.mark.parametrize("n,m,arity,R", [(3_000_000, 300, 8, 1_000_003), (1_000_000, 2652, 8, 262_144),
                                         (500_000, 100, 3, 77_777)])
def test_shards_synthetic_law(oracle_mod, n, m, arity, R):
    """The generator over shards draws node u's masks at the positions after
    the earlier shards' (a shifted key): the same tree as unsharded."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    d = 0.003 if m > 100 else 0.02
    dev = _sharded(R, lambda: BRWTDevice.synthetic(n, m, d, arity=arity, seed=17))
    assert dev.num_shards() == (n + R - 1) // R
    t = O.OracleTree.topdown(n, m, d, arity, 17)
    assert dev.num_relations() == t.num_relations()
    rows = np.random.default_rng(1).integers(0, n, 200_000).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    off_d, cols_d = dev.get_rows(rows)
    np.testing.assert_array_equal(off_d, off_o)
    np.testing.assert_array_equal(cols_d, cols_o)
    _same_tree(t.export(), dev.export())


def test_shards_synthetic_shaped(oracle_mod):
    """Greedy + relaxed shape (KIND_PACKT shards, k_traverse_ptw) over shards."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    rng = np.random.default_rng(5)
    dense = rng.random((4000, 300)) < 0.01
    shape = O.OracleTree.from_dense(dense, "greedy", 2, 10).export()
    n = 1_500_000
    dev = _sharded(400_000, lambda: BRWTDevice.synthetic_shaped(n, shape, 0.003, 7))
    assert dev.num_shards() == 4
    assert dev.traverse_kernel() == "k_traverse_ptw"
    t = O.OracleTree.topdown_shaped(n, shape, 0.003, 7)
    assert dev.num_relations() == t.num_relations()
    rows = rng.integers(0, n, 200_000).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    off_d, cols_d = dev.get_rows(rows)
    np.testing.assert_array_equal(off_d, off_o)
    np.testing.assert_array_equal(cols_d, cols_o)
    for j in (0, 150, 299):
        np.testing.assert_array_equal(dev.get_column(j), np.asarray(t.get_column(j), dtype=np.uint64))


def test_rows_beyond_2_32(oracle_mod):
    """4.5 B rows x 16 columns (3 shards of 2^31 rows) vs the streamed oracle:
    random rows over the whole range plus rows either side of every shard
    boundary and of 2^32; get_column over > 2^32 rows by its properties."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    n, m, d, arity, seed = 4_500_000_000, 16, 0.002, 4, 23
    dev = BRWTDevice.synthetic(n, m, d, arity=arity, seed=seed)
    assert dev.num_rows() == n and dev.num_shards() == 3
    rng = np.random.default_rng(7)
    edges = []
    for e in (2**31, 2**32, 2 * 2**31 + 1):
        edges += [e - 2, e - 1, e, e + 1]
    rows = np.concatenate([rng.integers(0, n, 300_000), edges, [0, n - 1]]).astype(np.uint64)
    off_o, cols_o = O.topdown_get_rows(n, m, d, arity, seed, rows)
    off_d, cols_d = dev.get_rows(rows)
    np.testing.assert_array_equal(off_d, off_o)
    np.testing.assert_array_equal(cols_d, cols_o)
    assert (rows >= 2**32).sum() > 10_000 and cols_o.size > 0
    # a column over the whole range: ascending, within range, beyond 2^32,
    # and membership agreeing with get_rows on a sample
    col = dev.get_column(5)
    assert col.size > 0 and np.all(np.diff(col.astype(np.int64)) > 0) and col[-1] < n and col[-1] >= 2**32
    assert abs(col.size - n * d) < 6 * np.sqrt(n * d)
    probe = np.concatenate([col[rng.integers(0, col.size, 2000)], rng.integers(0, n, 2000).astype(np.uint64)])
    off_p, cols_p = dev.get_rows(probe)
    has = np.array([5 in cols_p[off_p[i]:off_p[i + 1]] for i in range(len(probe))])
    np.testing.assert_array_equal(has, np.isin(probe, col))
    assert has[:2000].all()
