"""GPU parity of the ROW-RECORD layout (include/mbrwt.h "device layout",
csrc/rows.hip): contexts built with layout 'rows' (records only) and 'both'
against the CPU oracle -- bit-exact ordered CSR, point queries, columns,
count_labels and the V/L accounting -- on the reference's own grids
(test_BRWT.cpp:152-212, test_BRWT_optimizer.cpp:102-163), random basic /
greedy / relaxed trees, the C2 shape, the greedy + relax production shape,
every block size / rows-per-block choice, spilled and long records (the
direct pass), ranged builds and rows >= 2^32.
"""
import os

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def _dense_grid(kind, n, m):
    if kind == "zero":
        return np.zeros((n, m), dtype=bool)
    if kind == "one":
        return np.ones((n, m), dtype=bool)
    i = np.arange(n)[:, None]
    j = np.arange(m)[None, :]
    return ((i + 2 * j) % 2).astype(bool)  # test_BRWT.cpp:200


def _check_all(t, dev, rows, dense=None, columns=True):
    """Every row-record query against the oracle tree `t`."""
    off_o, cols_o = t.get_rows(rows)
    off_d, cols_d = dev.get_rows(rows)
    np.testing.assert_array_equal(off_d, off_o)
    np.testing.assert_array_equal(cols_d, cols_o)
    n, m = t.num_rows(), t.num_columns()
    rng = np.random.default_rng(n + 31 * m)
    k = min(4000, n * m)
    qr = rng.integers(0, n, k).astype(np.uint64)
    qc = rng.integers(0, m, k).astype(np.uint64)
    got = dev.get_batch(qr, qc)
    exp = np.array([t.get(int(r), int(c)) for r, c in zip(qr, qc)], dtype=np.uint8)
    np.testing.assert_array_equal(got, exp)
    if columns:
        for c in sorted(set(rng.integers(0, m, 6).tolist()) | {0, m - 1}):
            assert dev.get_column(c).tolist() == t.get_column(c)
    if dense is not None:
        for i in range(0, len(rows), max(1, len(rows) // 50)):
            r = int(rows[i])
            assert sorted(cols_d[off_d[i]:off_d[i + 1]].tolist()) == np.nonzero(dense[r])[0].tolist()
    return off_o, cols_o


def _count_labels(dev, rows):
    import torch
    rt = torch.from_numpy(np.ascontiguousarray(rows, dtype=np.uint64).view(np.int64)).cuda()
    ct = torch.zeros(max(1, dev.num_columns()), dtype=torch.int64, device="cuda")
    dev.count_labels_device(rt, ct)
    torch.cuda.synchronize()
    return ct.cpu().numpy().view(np.uint64)


@pytest.mark.parametrize("kind", ["zero", "one", "mixed"])
@pytest.mark.parametrize("build", [("basic", 2, 0), ("basic", 2, 2**64 - 1), ("greedy", 2, 0)])
def test_reference_grids_rows(oracle_mod, kind, build):
    """test_BRWT.cpp:152-212 / test_BRWT_optimizer.cpp:102-163 on row records."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice, MBRWTError, _lib as L
    part, arity, relax = build
    for n in range(1, 20):
        for m in range(1, 20):
            dense = _dense_grid(kind, n, m)
            t = O.OracleTree.from_dense(dense, part, arity, relax)
            ex = t.export()
            if m == 1:
                # a leaf root: outside the row-record layout (r06: nodes up to
                # 64 children wide -- relax without an arity bound -- are in)
                with pytest.raises(MBRWTError) as ei:
                    BRWTDevice.from_tree(ex, layout="rows")
                assert ei.value.status == L.MBRWT_ERR_UNSUPPORTED
                continue
            d = BRWTDevice.from_tree(ex, layout="rows")
            assert d.layout() == "rows"
            assert d.num_rows() == n and d.num_columns() == m and d.num_relations() == int(dense.sum())
            _check_all(t, d, np.arange(n, dtype=np.uint64), dense)


@pytest.mark.parametrize("n,m,d,part,arity,relax", [
    (5000, 40, 0.1, "basic", 2, 0),
    (5000, 40, 0.1, "basic", 3, 0),
    (5000, 40, 0.1, "greedy", 2, 0),
    (5000, 40, 0.1, "greedy", 2, 4),
    (3000, 100, 0.05, "basic", 8, 0),
    (3000, 100, 0.05, "basic", 2, 16),
    (2000, 200, 0.02, "basic", 16, 0),
    (6000, 200, 0.02, "greedy", 2, 10),   # the production shape (relax 10)
    (1000, 7, 1.0, "basic", 2, 0),        # dense rows
    (1000, 7, 0.0, "basic", 2, 0),        # rows without labels
])
@pytest.mark.parametrize("layout", ["rows", "both"])
def test_random_matrices_rows(oracle_mod, n, m, d, part, arity, relax, layout):
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    rng = np.random.default_rng(n * 7 + m)
    dense = rng.random((n, m)) < d
    t = O.OracleTree.from_dense(dense, part, arity, relax)
    dev = BRWTDevice.from_tree(t.export(), layout=layout)
    assert dev.layout() == layout
    assert dev.traverse_kernel() == "k_traverse_rows"
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 5000)]).astype(np.uint64)
    _check_all(t, dev, rows, dense)
    np.testing.assert_array_equal(_count_labels(dev, rows), dense[rows.astype(np.int64)].sum(axis=0))


@pytest.mark.parametrize("n,m,d,arity,levels", [
    (20000, 512, 0.02, 8, 2),      # root -> 8 -> 64 leaf parents
    (20000, 2652, 0.003, 8, 3),    # the Kingsford shape (C2-C4)
    (5000, 2652, 0.3, 8, 3),       # long records: spills and the direct pass
    (20000, 64, 0.05, 2, 5),       # binary, 5 internal levels
    (20000, 128, 0.05, 2, 0),      # binary, 6 levels: beyond the odometer (walk 6)
    (20000, 9, 0.2, 3, 1),         # the root's children are leaf parents
    (20000, 40, 0.1, 8, 1),
    (20000, 100, 0.05, 8, 2),      # 100 = 12 x 8 + 4: a short last group is still uniform
    (3000, 7, 1.0, 2, 0),          # singleton groups pass through: mixed depths
])
def test_odometer_walk(oracle_mod, build_env, n, m, d, arity, levels):
    """rows_walk_path / rows_walk_uni (one lock-step iteration per reached leaf
    parent, with / without the path table) and the general walk
    (MBRWT_OPT_ROWS_WALK = 6) return the oracle's CSR on uniform trees;
    non-uniform trees report 0 levels and keep the general walk (byte-mask
    records: the walks of terminal records are test_terminal_records')."""
    build_env("MBRWT_ROWS_CODE", 3)
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    rng = np.random.default_rng(n + m)
    dense = rng.random((n, m)) < d
    t = O.OracleTree.from_dense(dense, "basic", arity)
    dev = BRWTDevice.from_tree(t.export(), layout="rows")
    st = dev.rows_stats()
    ex = t.export()
    nc = np.asarray(ex["num_children"])
    assert st["uniform_levels"] == levels, (st, int(nc.max()))
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 20000)]).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    from genome_graph_annotation_amd import _lib as L
    # the path-table odometer, the tree odometer, the stack walks, the r03 odometer
    for walk in (0, 3, 4, 6, 7):
        dev.set_option(L.MBRWT_OPT_ROWS_WALK, walk)
        off_d, cols_d = dev.get_rows(rows)
        np.testing.assert_array_equal(off_d, off_o)
        np.testing.assert_array_equal(cols_d, cols_o)


@pytest.mark.parametrize("n,m,d,part,arity,relax", [
    (20000, 600, 0.01, "greedy", 2, 10),   # the reference's production shape (convert.sh:24): mixed depths
    (20000, 300, 0.05, "greedy", 2, 4),
    (20000, 256, 0.02, "greedy", 2, 0),    # binary greedy: 8+ internal levels
    (20000, 512, 0.02, "basic", 2, 0),     # binary, 9 internal levels: beyond the tree odometer
    (20000, 300, 0.02, "basic", 16, 0),    # two-byte masks
    (20000, 250, 0.05, "basic", 12, 0),    # arity 12: two-byte masks, mixed depths
    (4000, 300, 0.4, "greedy", 2, 10),     # long records: spills and the direct pass
    (3000, 7, 1.0, "basic", 2, 0),         # singleton groups pass through
])
def test_tree_odometer(oracle_mod, build_env, n, m, d, part, arity, relax):
    """rows_walk_tree (the default on non-uniform trees: one lock-step
    iteration per reached leaf parent or leaf, leaf parents at any depth,
    non-consecutive leaf parents walked as internal nodes, masks up to 16
    bits) returns the oracle's CSR, as do the stack walks it replaced."""
    build_env("MBRWT_ROWS_CODE", 3)  # (byte masks: the odometers)
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    from genome_graph_annotation_amd import _lib as L
    rng = np.random.default_rng(n + m + arity)
    dense = rng.random((n, m)) < d
    t = O.OracleTree.from_dense(dense, part, arity, relax)
    dev = BRWTDevice.from_tree(t.export(), layout="rows")
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 20000)]).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    for walk in (0, 3, 4, 6):
        dev.set_option(L.MBRWT_OPT_ROWS_WALK, walk)
        off_d, cols_d = dev.get_rows(rows)
        np.testing.assert_array_equal(off_d, off_o)
        np.testing.assert_array_equal(cols_d, cols_o)


def test_auto_layout(oracle_mod, build_env):
    """The library default (MBRWT_LAYOUT_AUTO): row records for every tree
    within their limits whose records fit one block request per row; the
    per-node images for a one-column tree, nodes wider than 64 children,
    records too long for the block layout (dense rows), or MBRWT_LAYOUT=nodes."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    rng = np.random.default_rng(12)
    sparse = rng.random((5000, 300)) < 0.01
    for part, arity, relax in [("basic", 8, 0), ("greedy", 2, 10), ("basic", 2, 0)]:
        t = O.OracleTree.from_dense(sparse, part, arity, relax)
        d = BRWTDevice.from_tree(t.export())
        assert d.layout() == "rows" and d.traverse_kernel() == "k_traverse_rows"
        _check_all(t, d, np.arange(5000, dtype=np.uint64), sparse, columns=False)
    assert BRWTDevice.synthetic(200_000, 2652, 0.003, 8, 42).layout() == "rows"
    W = (5000 + 63) // 64
    words = [np.pad(np.packbits(sparse[:, j], bitorder="little"), (0, 8 * W - (5000 + 7) // 8)).view(np.uint64)
             for j in range(300)]
    assert BRWTDevice.from_columns(words, 5000, 8).layout() == "rows"
    one = O.OracleTree.from_dense(sparse[:, :1], "basic", 2)
    assert BRWTDevice.from_tree(one.export()).layout() == "nodes"
    dense = rng.random((3000, 2652)) < 0.3  # ~800 labels per row: long records
    td = O.OracleTree.from_dense(dense, "basic", 8)
    dd = BRWTDevice.from_tree(td.export())  # a uniform tree: variable-length records
    assert dd.layout() == "rows" and dd.rows_stats()["variable"]
    _check_all(td, dd, np.arange(0, 3000, 7, dtype=np.uint64), dense, columns=False)
    tg = O.OracleTree.from_dense(dense, "greedy", 2, 10)  # records longer than a block, not uniform: the node images
    dg = BRWTDevice.from_tree(tg.export())
    assert dg.layout() == "nodes"
    _check_all(tg, dg, np.arange(0, 3000, 7, dtype=np.uint64), dense, columns=False)
    build_env("MBRWT_LAYOUT", "nodes")
    assert BRWTDevice.from_tree(O.OracleTree.from_dense(sparse, "basic", 8).export()).layout() == "nodes"


@pytest.mark.parametrize("n,m,d,part,arity,relax,max_arity", [
    (500, 64, 0.1, "basic", 33, 0, 33),                # one node of 33 children above one of 31
    (500, 64, 0.1, "basic", 64, 0, 64),                # one level: the root holds 64 leaves
    (5000, 200, 0.05, "greedy", 2, 2**64 - 1, 25),     # relax without an arity bound
    (5000, 300, 0.1, "greedy", 2, 2**64 - 1, 37),      # (test_BRWT_optimizer.cpp:102-163)
    (4000, 400, 0.05, "greedy", 2, 2**64 - 1, 50),
])
def test_wide_nodes_rows(oracle_mod, n, m, d, part, arity, relax, max_arity):
    """Row records over nodes up to 64 children wide (r06; 16 before): masks
    of up to eight bytes, walked by the tree odometer and the one-lane walks;
    the library default (AUTO) takes them; every query and the export back
    into index columns against the oracle."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    rng = np.random.default_rng(n + m)
    dense = rng.random((n, m)) < d
    t = O.OracleTree.from_dense(dense, part, arity, relax)
    ex = t.export()
    assert int(np.asarray(ex["num_children"]).max()) == max_arity
    dev = BRWTDevice.from_tree(ex)
    assert dev.layout() == "rows" and dev.traverse_kernel() == "k_traverse_rows"
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 20000)]).astype(np.uint64)
    _check_all(t, dev, rows, dense)
    np.testing.assert_array_equal(_count_labels(dev, rows), dense[rows.astype(np.int64)].sum(axis=0))
    back = dev.export()
    for k in ("num_children", "first_child", "leaf_column"):
        np.testing.assert_array_equal(np.asarray(back[k]), np.asarray(ex[k]))


@pytest.mark.parametrize("n,m,d,part,arity,relax", [
    (20000, 2652, 0.003, "basic", 8, 0),     # the Kingsford shape
    (4000, 300, 0.4, "greedy", 2, 10),       # dense rows: direct tiles and long records in the compaction
])
def test_compact_cus_option(oracle_mod, n, m, d, part, arity, relax):
    """MBRWT_OPT_COMPACT_CUS (r06): the compaction on a CU-masked stream
    between two events returns the same CSR, on a context and its clone,
    through the host and the device entry points; out-of-range values are
    rejected."""
    import torch
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice, MBRWTError, _lib as L
    rng = np.random.default_rng(n + m)
    dense = rng.random((n, m)) < d
    t = O.OracleTree.from_dense(dense, part, arity, relax)
    dev = BRWTDevice.from_tree(t.export())
    assert dev.layout() == "rows"
    twin = dev.clone()
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 20000)]).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    for cus in (4, 16, 31, 0):
        for q in (dev, twin):
            q.set_option(L.MBRWT_OPT_COMPACT_CUS, cus)
            off_d, cols_d = q.get_rows(rows)
            np.testing.assert_array_equal(off_d, off_o)
            np.testing.assert_array_equal(cols_d, cols_o)
    dev.set_option(L.MBRWT_OPT_COMPACT_CUS, 8)
    s = torch.cuda.Stream()
    rt = torch.from_numpy(rows.view(np.int64)).cuda()
    ot = torch.zeros(len(rows) + 1, dtype=torch.int64, device="cuda")
    ct = torch.zeros(max(1, len(cols_o)), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    assert dev.get_rows_device(rt, ot, ct, s.cuda_stream) == len(cols_o)
    s.synchronize()
    np.testing.assert_array_equal(ot.cpu().numpy().view(np.uint64), off_o)
    np.testing.assert_array_equal(ct.cpu().numpy().view(np.uint32)[:len(cols_o)], cols_o)
    for bad in (-1, 32):
        with pytest.raises(MBRWTError):
            dev.set_option(L.MBRWT_OPT_COMPACT_CUS, bad)


@pytest.mark.parametrize("m,arity", [(40000, 8), (33000, 6), (65536, 16)])
def test_many_columns_rows(oracle_mod, m, arity):
    """Row records over 2^15 .. 2^16 columns (r06; < 2^15 before): the RWT
    table's leaves carry 16-bit columns, the labels stay u16 in the stage."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    n = 1500
    rng = np.random.default_rng(m)
    # (about 3.5 labels a row: records of one block request per row, which
    # AUTO takes -- 12 a row at 40,000 columns made it choose the node images)
    dense = rng.random((n, m)) < 3.0 / m
    dense[:, m - 1] |= rng.random(n) < 0.5  # (the last column in use)
    t = O.OracleTree.from_dense(dense, "basic", arity)
    dev = BRWTDevice.from_tree(t.export())
    assert dev.layout() == "rows" and dev.traverse_kernel() == "k_traverse_rows"
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 5000)]).astype(np.uint64)
    _check_all(t, dev, rows, dense)
    np.testing.assert_array_equal(_count_labels(dev, rows), dense[rows.astype(np.int64)].sum(axis=0))


@pytest.mark.parametrize("m,arity", [(70000, 8), (33000, 2)])
def test_columns_limit(oracle_mod, m, arity):
    """Beyond 2^16 columns the u16 label stage no longer holds a label, and a
    walk table (RWT2, one entry per child of every internal node above the
    leaf parents) beyond the 8,192 words staged in LDS -- 33,000 columns
    under a binary tree -- has no record walk: the node layout answers."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice, MBRWTError, _lib as L
    n = 600
    rng = np.random.default_rng(3)
    dense = rng.random((n, m)) < 5.0 / m
    dense[:, m - 1] = True
    t = O.OracleTree.from_dense(dense, "basic", arity)
    with pytest.raises(MBRWTError) as ei:
        BRWTDevice.from_tree(t.export(), layout="rows")
    assert ei.value.status == L.MBRWT_ERR_UNSUPPORTED
    d = BRWTDevice.from_tree(t.export())
    assert d.layout() == "nodes"
    _check_all(t, d, np.arange(n, dtype=np.uint64), dense, columns=False)


def test_arity_limit(oracle_mod):
    """Nodes wider than 64 children (relax without an arity bound on a dense
    matrix: 193 children under one node) are outside every layout of this
    build (masks are held in 64 bits): a clean MBRWT_ERR_UNSUPPORTED."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice, MBRWTError, _lib as L
    dense = np.random.default_rng(2).random((3000, 200)) < 0.2
    t = O.OracleTree.from_dense(dense, "greedy", 2, 2**64 - 1)
    assert int(np.asarray(t.export()["num_children"]).max()) > 64
    for layout in ("rows", None):
        with pytest.raises(MBRWTError) as ei:
            BRWTDevice.from_tree(t.export(), layout=layout) if layout else BRWTDevice.from_tree(t.export())
        assert ei.value.status == L.MBRWT_ERR_UNSUPPORTED


@pytest.mark.parametrize("bs", ["64,1", "64,2", "64,3", "64,5", "64,8", "128,1", "128,3", "128,7", "128,15"])
def test_every_block_shape(oracle_mod, bs, build_env):
    """Every (block bytes, rows per block) the builder may pick -- spills,
    long records and the direct pass included -- answers like the oracle."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    build_env("MBRWT_ROWS_BS", bs)
    # (byte masks: a fully dense row's terminal fields outgrow a 64-byte
    # block where its masks do not, and AUTO then takes the variable-length
    # records -- terminal records' spills and long rows: test_terminal_records)
    build_env("MBRWT_ROWS_CODE", 3)
    rng = np.random.default_rng(5)
    n, m = 30000, 300
    # rows of very different lengths: most sparse, some dense (long records)
    u = rng.random(n)
    p = np.where(u < 0.005, 1.0, np.where(u < 0.025, 0.5, 0.01))
    dense = rng.random((n, m)) < p[:, None]
    for part, arity, relax in [("basic", 8, 0), ("greedy", 2, 10)]:
        t = O.OracleTree.from_dense(dense, part, arity, relax)
        dev = BRWTDevice.from_tree(t.export(), layout="rows")
        st = dev.rows_stats()
        B, S = (int(x) for x in bs.split(","))
        assert (st["block_bytes"], st["rows_per_block"]) == (B, S)
        rows = np.concatenate([np.arange(n), rng.integers(0, n, 20000)]).astype(np.uint64)
        _check_all(t, dev, rows, dense, columns=False)


def test_synthetic_c2_shape_rows(oracle_mod):
    """C2 (1 M x 2,652, d = 0.3 %, arity 8) generated on the device, turned
    into row records; the whole batch, V/L and count_labels against the
    oracle's independent generator."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    n, m, d = 1_000_000, 2652, 0.003
    t = O.OracleTree.topdown(n, m, d, 8, 42)
    rows = np.random.default_rng(42).integers(0, n, 300_000).astype(np.uint64)
    both = BRWTDevice.synthetic(n, m, d, 8, 42, layout="both")
    rec = BRWTDevice.synthetic(n, m, d, 8, 42, layout="rows")
    assert rec.device_bytes() < both.device_bytes()
    off_o, cols_o = t.get_rows(rows)
    for dev in (both, rec):
        off_d, cols_d = dev.get_rows(rows)
        np.testing.assert_array_equal(off_d, off_o)
        np.testing.assert_array_equal(cols_d, cols_o)
    import torch
    rt = torch.from_numpy(rows.view(np.int64)).cuda()
    v_rec = rec.count_work_device(rt)
    nodes = BRWTDevice.synthetic(n, m, d, 8, 42, layout="nodes")
    v_nodes = nodes.count_work_device(rt)
    assert v_rec == v_nodes, (v_rec, v_nodes)
    np.testing.assert_array_equal(_count_labels(rec, rows), np.bincount(cols_o, minlength=m))
    for c in (0, 1, 1000, m - 1):
        assert rec.get_column(c).tolist() == t.get_column(c)


def test_greedy_relax_shape_rows(oracle_mod):
    """The production shape (greedy + relax 10 from C2's columns, the
    reference's build scripts) under the synthetic law, as row records."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    dense = np.random.default_rng(11).random((20000, 2652)) < 0.003
    shape = O.OracleTree.from_dense(dense, "greedy", 2, 10).export()
    n = 400_000
    dev = BRWTDevice.synthetic_shaped(n, shape, 0.003, 7, layout="rows")
    t = O.OracleTree.topdown_shaped(n, shape, 0.003, 7)
    rows = np.random.default_rng(3).integers(0, n, 200_000).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    off_d, cols_d = dev.get_rows(rows)
    np.testing.assert_array_equal(off_d, off_o)
    np.testing.assert_array_equal(cols_d, cols_o)


def test_ranged_build(oracle_mod, build_env):
    """Layout rows built one range of rows at a time (synthetic law across
    the ranges, and a tree description sliced per range)."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    build_env("MBRWT_ROWS_RANGE", "360360")
    n, m, d = 1_500_000, 700, 0.004
    dev = BRWTDevice.synthetic(n, m, d, 8, 9, layout="rows")
    t = O.OracleTree.topdown(n, m, d, 8, 9)
    rows = np.concatenate([np.arange(360350, 360370), np.arange(720710, 720730),
                           np.random.default_rng(1).integers(0, n, 200_000)]).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    off_d, cols_d = dev.get_rows(rows)
    np.testing.assert_array_equal(off_d, off_o)
    np.testing.assert_array_equal(cols_d, cols_o)
    # from a description (slice_desc per range)
    rng = np.random.default_rng(2)
    dense = rng.random((800_000, 40)) < 0.05
    t2 = O.OracleTree.from_dense(dense, "greedy", 2, 4)
    dev2 = BRWTDevice.from_tree(t2.export(), layout="rows")
    _check_all(t2, dev2, rng.integers(0, 800_000, 100_000).astype(np.uint64), dense, columns=False)


def test_errors_and_capacity_rows(oracle_mod):
    O = oracle_mod
    import ctypes as C
    from genome_graph_annotation_amd import BRWTDevice, MBRWTError, _lib as L
    rng = np.random.default_rng(3)
    dense = rng.random((100, 20)) < 0.5
    t = O.OracleTree.from_dense(dense, "basic", 4)
    d = BRWTDevice.from_tree(t.export(), layout="rows")
    with pytest.raises(MBRWTError) as ei:
        d.get_rows(np.array([0, 100], dtype=np.uint64))
    assert ei.value.status == L.MBRWT_ERR_RANGE
    with pytest.raises(MBRWTError):
        d.get_batch([0], [20])
    with pytest.raises(MBRWTError):
        d.get_column(20)
    # capacity retry protocol
    rows = np.arange(100, dtype=np.uint64)
    off = np.zeros(101, dtype=np.uint64)
    cols = np.zeros(5, dtype=np.uint32)
    need = C.c_uint64(0)
    rc = L.lib().mbrwt_get_rows(d._h, rows.ctypes.data_as(L.u64p), 100, off.ctypes.data_as(L.u64p),
                                cols.ctypes.data_as(L.u32p), 5, C.byref(need))
    assert rc == L.MBRWT_ERR_CAPACITY and need.value == int(dense.sum())
    off_d, cols_d = d.get_rows(rows)
    off_o, cols_o = t.get_rows(rows)
    np.testing.assert_array_equal(off_d, off_o)
    np.testing.assert_array_equal(cols_d, cols_o)
    e, c2 = d.get_rows(np.zeros(0, dtype=np.uint64))
    assert e.tolist() == [0] and len(c2) == 0


@pytest.mark.parametrize("shape", ["uniform", "greedy", "long"])
def test_async_capacity_boundary_and_batches(oracle_mod, shape):
    """The asynchronous row-record call on batches of 1 .. 31k tiles (uniform,
    greedy + relax, and long records: direct tiles, spills): the oracle's
    CSR; the capacity boundary (cap = total is enough, total - 1 reports
    MBRWT_ERR_CAPACITY and writes nothing past the capacity); a row out of
    range in the middle of the batch; many calls back to back through one
    status block.  (r06: also the one-pass traversal's test while it existed,
    profiles/r06/v01_one_pass.)"""
    O = oracle_mod
    import torch
    from genome_graph_annotation_amd import BRWTDevice, _lib as L
    rng = np.random.default_rng(17)
    n, m, d, part, arity, relax = {
        "uniform": (30000, 2652, 0.003, "basic", 8, 0),
        "greedy": (30000, 600, 0.01, "greedy", 2, 10),
        "long": (3000, 2652, 0.3, "basic", 8, 0),       # direct tiles, spilled and long records
    }[shape]
    dense = rng.random((n, m)) < d
    t = O.OracleTree.from_dense(dense, part, arity, relax)
    dev = BRWTDevice.from_tree(t.export(), layout="rows")
    s = torch.cuda.current_stream().cuda_stream
    st = torch.zeros(3, dtype=torch.int64, device="cuda")
    sizes = (1, 64, 65, 4097, 2_000_000) if shape != "long" else (1, 64, 65, 4097, 60_000)
    for k in sizes:
        rows = rng.integers(0, n, k).astype(np.uint64)
        off_o, cols_o = t.get_rows(rows)
        tot = len(cols_o)
        rt = torch.from_numpy(rows.view(np.int64)).cuda()
        ot = torch.empty(k + 1, dtype=torch.int64, device="cuda")
        ct = torch.full((tot + 64,), -1, dtype=torch.int32, device="cuda")
        for cap in (tot, max(0, tot - 1)):
            st.zero_()
            ct.fill_(-1)
            dev.get_rows_device_async(rt, ot, ct[:cap], st, s)
            torch.cuda.synchronize()
            need, status, sticky = st.cpu().tolist()
            assert need == tot
            if cap >= tot:
                assert status == L.MBRWT_OK and sticky == 1 << L.MBRWT_OK
                np.testing.assert_array_equal(ot.cpu().numpy().view(np.uint64), off_o)
                np.testing.assert_array_equal(ct[:tot].cpu().numpy().view(np.uint32), cols_o)
            else:
                assert status == L.MBRWT_ERR_CAPACITY and sticky == 1 << L.MBRWT_ERR_CAPACITY
            assert (ct[cap:] == -1).all(), "a label written past the capacity"
        # a row out of range in the middle of the batch
        if k > 64:
            bad = rows.copy()
            bad[k // 2] = n
            bt = torch.from_numpy(bad.view(np.int64)).cuda()
            st.zero_()
            ct = torch.empty(tot + 64, dtype=torch.int32, device="cuda")
            dev.get_rows_device_async(bt, ot, ct, st, s)
            torch.cuda.synchronize()
            assert st.cpu().tolist()[1] == L.MBRWT_ERR_RANGE
    # many asynchronous calls back to back on one context
    rows = rng.integers(0, n, 100_000).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    rt = torch.from_numpy(rows.view(np.int64)).cuda()
    ot = torch.empty(len(rows) + 1, dtype=torch.int64, device="cuda")
    ct = torch.empty(len(cols_o) + 1, dtype=torch.int32, device="cuda")
    st.zero_()
    for _ in range(50):
        dev.get_rows_device_async(rt, ot, ct, st, s)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [len(cols_o), L.MBRWT_OK, 1 << L.MBRWT_OK]
    np.testing.assert_array_equal(ot.cpu().numpy().view(np.uint64), off_o)
    np.testing.assert_array_equal(ct[:len(cols_o)].cpu().numpy().view(np.uint32), cols_o)


# ---- nibble-coded masks (r06, MBRWT_BUILD_ROWS_CODE = 1) ------------

@pytest.mark.parametrize("n,m,d,arity", [
    (20000, 2652, 0.003, 8),   # the Kingsford shape (C2-C4)
    (20000, 512, 0.02, 8),
    (5000, 2652, 0.3, 8),      # dense rows: multi-bit masks, spills, long records, direct tiles
    (20000, 64, 0.05, 2),      # binary, 5 internal levels
    (20000, 100, 0.05, 8),     # a short last group
    (20000, 9, 0.2, 3),        # the root's children are leaf parents
    (3000, 40, 0.0, 8),        # rows without labels
])
def test_nibble_codes(oracle_mod, build_env, n, m, d, arity):
    """Row records whose masks are nibble codes: every query (ordered CSR,
    point queries, columns, count_labels, the V/L accounting, the async call)
    against the oracle and against the byte-coded image of the same tree,
    and the image exported back into the reference's index columns."""
    O = oracle_mod
    import torch
    from genome_graph_annotation_amd import BRWTDevice, _lib as L
    rng = np.random.default_rng(n + m + arity)
    dense = rng.random((n, m)) < d
    t = O.OracleTree.from_dense(dense, "basic", arity)
    ex = t.export()
    build_env("MBRWT_ROWS_CODE", 3)  # (byte masks: the baseline)
    plain = BRWTDevice.from_tree(ex, layout="rows")
    build_env("MBRWT_ROWS_CODE", 1)
    dev = BRWTDevice.from_tree(ex, layout="rows")
    st, sp = dev.rows_stats(), plain.rows_stats()
    assert not sp["nibble_codes"] and (sp["uniform_levels"] > 0 or not st["nibble_codes"]), (st, sp)
    # nibble codes where they shrink the records (bytes kept otherwise: dense rows)
    assert st["record_bytes"] <= sp["record_bytes"], (st, sp)
    assert st["nibble_codes"] == (st["record_bytes"] < sp["record_bytes"]), (st, sp)
    if (m, d) == (2652, 0.003):
        assert st["nibble_codes"] and st["record_bytes"] < 0.8 * sp["record_bytes"], (st, sp)
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 20000)]).astype(np.uint64)
    off_o, cols_o = _check_all(t, dev, rows, dense)
    np.testing.assert_array_equal(_count_labels(dev, rows), _count_labels(plain, rows))
    rt = torch.from_numpy(rows.view(np.int64)).cuda()
    assert dev.count_work_device(rt) == plain.count_work_device(rt)
    # the asynchronous call
    s = torch.cuda.current_stream().cuda_stream
    stt = torch.zeros(3, dtype=torch.int64, device="cuda")
    ot = torch.empty(len(rows) + 1, dtype=torch.int64, device="cuda")
    ct = torch.empty(len(cols_o) + 1, dtype=torch.int32, device="cuda")
    dev.get_rows_device_async(rt, ot, ct, stt, s)
    torch.cuda.synchronize()
    assert stt.cpu().tolist() == [len(cols_o), L.MBRWT_OK, 1 << L.MBRWT_OK]
    np.testing.assert_array_equal(ot.cpu().numpy().view(np.uint64), off_o)
    # the reference's index columns read back from the nibble-coded records
    back = dev.export()
    for k in ("num_children", "first_child", "leaf_column"):
        np.testing.assert_array_equal(np.asarray(back[k]), np.asarray(ex[k]))
    again = BRWTDevice.from_tree(back, layout="rows")
    off_a, cols_a = again.get_rows(rows)
    np.testing.assert_array_equal(off_a, off_o)
    np.testing.assert_array_equal(cols_a, cols_o)


@pytest.mark.parametrize("n,m,d,part,arity,relax", [
    (20000, 2652, 0.003, "basic", 8, 0),      # the Kingsford shape (uniform)
    (20000, 600, 0.01, "greedy", 2, 10),      # the reference's production shape: mixed depths, listed leaf parents
    (20000, 300, 0.05, "greedy", 2, 4),
    (20000, 256, 0.02, "greedy", 2, 0),       # binary greedy: 8+ internal levels
    (20000, 250, 0.05, "basic", 12, 0),       # two-byte masks, mixed depths
    (20000, 9, 0.2, "basic", 3, 0),           # the root's children are leaf parents
    (2000, 12, 0.3, "basic", 16, 0),          # a one-level tree: the root is the only terminal
    (3000, 7, 1.0, "basic", 2, 0),            # singleton groups: leaves beside internal nodes
    (4000, 300, 0.4, "greedy", 2, 10),        # dense rows: long records, direct tiles (or bytes kept)
])
def test_terminal_records(oracle_mod, build_env, n, m, d, part, arity, relax):
    """Terminal records (MBRWT_BUILD_ROWS_CODE = 2; the AUTO default where
    smaller): each row as the leaf parents and leaves its descent reaches, in
    pre-order -- every query (ordered CSR, point queries, columns,
    count_labels, the V/L accounting, the async call) against the oracle and
    the byte-mask image of the same tree, and the export back into the
    reference's index columns."""
    O = oracle_mod
    import torch
    from genome_graph_annotation_amd import BRWTDevice, MBRWTError, _lib as L
    rng = np.random.default_rng(n + m + arity)
    dense = rng.random((n, m)) < d
    t = O.OracleTree.from_dense(dense, part, arity, relax)
    ex = t.export()
    build_env("MBRWT_ROWS_CODE", 3)  # (byte masks: the baseline)
    plain = BRWTDevice.from_tree(ex, layout="rows")
    build_env("MBRWT_ROWS_CODE", 2)
    dev = BRWTDevice.from_tree(ex, layout="rows")
    st, sp = dev.rows_stats(), plain.rows_stats()
    assert not sp["terminal_records"]
    # terminal fields where they shrink the records (bytes kept otherwise)
    assert st["record_bytes"] <= sp["record_bytes"], (st, sp)
    assert st["terminal_records"] == (st["record_bytes"] < sp["record_bytes"]), (st, sp)
    if d <= 0.05:
        assert st["terminal_records"], (st, sp)
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 20000)]).astype(np.uint64)
    off_o, cols_o = _check_all(t, dev, rows, dense)
    np.testing.assert_array_equal(_count_labels(dev, rows), _count_labels(plain, rows))
    rt = torch.from_numpy(rows.view(np.int64)).cuda()
    s = torch.cuda.current_stream().cuda_stream
    stt = torch.zeros(3, dtype=torch.int64, device="cuda")
    ot = torch.empty(len(rows) + 1, dtype=torch.int64, device="cuda")
    ct = torch.empty(len(cols_o) + 1, dtype=torch.int32, device="cuda")
    dev.get_rows_device_async(rt, ot, ct, stt, s)
    torch.cuda.synchronize()
    assert stt.cpu().tolist() == [len(cols_o), L.MBRWT_OK, 1 << L.MBRWT_OK]
    np.testing.assert_array_equal(ot.cpu().numpy().view(np.uint64), off_o)
    np.testing.assert_array_equal(ct.cpu().numpy().view(np.uint32)[:len(cols_o)], cols_o)
    # the V accounting (the terminals' ancestor chains) and the export (the
    # index columns rebuilt from the terminals) equal the byte records'
    assert dev.count_work_device(rt) == plain.count_work_device(rt)
    back = dev.export()
    for k in ("num_children", "first_child", "leaf_column"):
        np.testing.assert_array_equal(np.asarray(back[k]), np.asarray(ex[k]))
    again = BRWTDevice.from_tree(back, layout="rows")
    off_a, cols_a = again.get_rows(rows)
    np.testing.assert_array_equal(off_a, off_o)
    np.testing.assert_array_equal(cols_a, cols_o)
    # out-of-range rows still report MBRWT_ERR_RANGE
    with pytest.raises(MBRWTError) as ei:
        dev.get_rows(np.array([n], dtype=np.uint64))
    assert ei.value.status == L.MBRWT_ERR_RANGE


def test_terminal_records_kingsford_synthetic(oracle_mod, build_env):
    """The C2 shape generated on the device with terminal records: the whole
    batch against the oracle's independent generator and the image against
    the byte-coded one."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    n, m, d = 1_000_000, 2652, 0.003
    build_env("MBRWT_ROWS_CODE", 3)
    plain = BRWTDevice.synthetic(n, m, d, 8, 42, layout="rows")
    build_env("MBRWT_ROWS_CODE", 2)
    dev = BRWTDevice.synthetic(n, m, d, 8, 42, layout="rows")
    st = dev.rows_stats()
    assert st["terminal_records"], st
    assert dev.device_bytes() < plain.device_bytes(), (dev.device_bytes(), plain.device_bytes())
    t = O.OracleTree.topdown(n, m, d, 8, 42)
    rows = np.random.default_rng(42).integers(0, n, 300_000).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    off_d, cols_d = dev.get_rows(rows)
    np.testing.assert_array_equal(off_d, off_o)
    np.testing.assert_array_equal(cols_d, cols_o)


def test_nibble_codes_kingsford_synthetic(oracle_mod, build_env):
    """The C2 shape generated on the device with nibble-coded records: the
    whole batch against the oracle's independent generator, three rows per
    64-byte block, and the image at most 0.75x the byte-coded one."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    n, m, d = 1_000_000, 2652, 0.003
    build_env("MBRWT_ROWS_CODE", 3)
    plain = BRWTDevice.synthetic(n, m, d, 8, 42, layout="rows")
    build_env("MBRWT_ROWS_CODE", 1)
    dev = BRWTDevice.synthetic(n, m, d, 8, 42, layout="rows")
    st = dev.rows_stats()
    assert st["nibble_codes"] and st["block_bytes"] == 64 and st["rows_per_block"] >= 3, st
    assert dev.device_bytes() <= 0.75 * plain.device_bytes(), (dev.device_bytes(), plain.device_bytes())
    t = O.OracleTree.topdown(n, m, d, 8, 42)
    rows = np.random.default_rng(42).integers(0, n, 300_000).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    off_d, cols_d = dev.get_rows(rows)
    np.testing.assert_array_equal(off_d, off_o)
    np.testing.assert_array_equal(cols_d, cols_o)
    for c in (0, 1, 1000, m - 1):
        assert dev.get_column(c).tolist() == t.get_column(c)


def test_classify_on_rows(oracle_mod):
    """get_labels / get_top_labels batches (classify) over row records, against
    the reference's semantics applied to the oracle's rows
    (annotate_static.cpp:71-94, annotate.cpp:57-83)."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    from test_gpu_parity import _ref_get_labels, _ref_top_labels
    rng = np.random.default_rng(8)
    n, m = 20000, 300
    dense = rng.random((n, m)) < 0.03
    t = O.OracleTree.from_dense(dense, "basic", 8)
    dev = BRWTDevice.from_tree(t.export(), layout="rows")
    assert dev.layout() == "rows"
    lens = rng.integers(0, 40, 1000)
    roff = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    rows = rng.integers(0, n, int(roff[-1])).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    for ratio in (0.0, 0.5, 1.0):
        want = _ref_get_labels(off_o, cols_o, roff, m, ratio)
        got = dev.get_labels_batch(rows, roff, ratio)
        for x, y in zip(got, want):
            np.testing.assert_array_equal(x, y)
    for num_top in (5, 2**64 - 1):
        want = _ref_top_labels(off_o, cols_o, roff, m, num_top)
        got = dev.get_top_labels_batch(rows, roff, num_top)
        for x, y in zip(got, want):
            np.testing.assert_array_equal(x, y)


@pytest.mark.slow
def test_rows_beyond_2_32_rows(oracle_mod):
    """Rows >= 2^32 without row shards: a 4.5 B-row x 16-column tree as row
    records (ranged build), against the streamed oracle."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    n, m, d = 4_500_000_000, 16, 0.01
    dev = BRWTDevice.synthetic(n, m, d, 4, 5, layout="rows")
    assert dev.num_shards() == 1 and dev.layout() == "rows"
    rng = np.random.default_rng(4)
    edges = []
    for e in (2**31, 2**32, 3 * 2**31, n):
        edges += list(range(e - 8, min(e + 8, n)))
    rows = np.concatenate([np.array(edges), rng.integers(0, n, 300_000)]).astype(np.uint64)
    off_o, cols_o = O.topdown_get_rows(n, m, d, 4, 5, rows)
    off_d, cols_d = dev.get_rows(rows)
    np.testing.assert_array_equal(off_d, off_o)
    np.testing.assert_array_equal(cols_d, cols_o)


@pytest.mark.parametrize("layout", ["rows", "nodes"])
def test_get_rows_device_async(oracle_mod, layout):
    """mbrwt_get_rows_device_async: several batches enqueued back to back with
    no host synchronisation, the status block {needed, status, sticky bits}
    read once at the end; capacity and range errors reported through it."""
    O = oracle_mod
    import torch
    from genome_graph_annotation_amd import BRWTDevice, _lib as L
    rng = np.random.default_rng(11)
    n, m = 30000, 200
    dense = rng.random((n, m)) < 0.04
    t = O.OracleTree.from_dense(dense, "basic", 8)
    d = BRWTDevice.from_tree(t.export(), layout=layout)
    s = torch.cuda.current_stream().cuda_stream
    st = torch.zeros(3, dtype=torch.int64, device="cuda")
    outs = []
    for k in (1, 63, 64, 65, 5000, 40000):
        rows = rng.integers(0, n, k).astype(np.uint64)
        rt = torch.from_numpy(rows.view(np.int64)).cuda()
        ot = torch.empty(k + 1, dtype=torch.int64, device="cuda")
        ct = torch.empty(k * m // 10 + 64, dtype=torch.int32, device="cuda")
        d.get_rows_device_async(rt, ot, ct, st, s)
        outs.append((rows, ot, ct, st.clone()))
    torch.cuda.synchronize()
    for rows, ot, ct, st_k in outs:
        off_o, cols_o = t.get_rows(rows)
        need, status, sticky = st_k.cpu().tolist()
        assert status == L.MBRWT_OK and need == len(cols_o)
        assert sticky == 1 << L.MBRWT_OK
        np.testing.assert_array_equal(ot.cpu().numpy().view(np.uint64), off_o)
        np.testing.assert_array_equal(ct[:need].cpu().numpy().view(np.uint32), cols_o)
    rows = rng.integers(0, n, 3000).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    rt = torch.from_numpy(rows.view(np.int64)).cuda()
    ot = torch.empty(3001, dtype=torch.int64, device="cuda")
    small = torch.empty(5, dtype=torch.int32, device="cuda")
    st.zero_()
    d.get_rows_device_async(rt, ot, small, st, s)
    torch.cuda.synchronize()
    need, status, sticky = st.cpu().tolist()
    assert status == L.MBRWT_ERR_CAPACITY and need == len(cols_o)
    assert sticky & (1 << L.MBRWT_ERR_CAPACITY)
    bad = torch.tensor([0, n], dtype=torch.int64, device="cuda")
    ot2 = torch.empty(3, dtype=torch.int64, device="cuda")
    ct2 = torch.empty(1000, dtype=torch.int32, device="cuda")
    st.zero_()
    d.get_rows_device_async(bad, ot2, ct2, st, s)
    torch.cuda.synchronize()
    assert st.cpu().tolist()[1] == L.MBRWT_ERR_RANGE
    # a good call after the errors
    ct = torch.empty(len(cols_o) + 1, dtype=torch.int32, device="cuda")
    st.zero_()
    d.get_rows_device_async(rt, ot, ct, st, s)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [len(cols_o), L.MBRWT_OK, 1 << L.MBRWT_OK]
    np.testing.assert_array_equal(ct[:len(cols_o)].cpu().numpy().view(np.uint32), cols_o)


# ---- variable-length records (csrc/rows_var.hip; dense rows) ------------------

@pytest.mark.parametrize("n,m,d,arity", [
    (5000, 3173, 0.038, 8),   # the RefSeq shape (C3), reduced rows
    (4000, 700, 0.2, 8),
    (3000, 64, 0.3, 2),       # binary, 5 levels above the leaf parents
    (3000, 45, 0.5, 3),
    (2000, 100, 0.05, 8),     # 100 = 12 x 8 + 4: a short last leaf parent
    (2000, 300, 0.0, 8),      # no labels at all: no records
    (1000, 2652, 0.003, 8),   # sparse (most rows without a record)
])
@pytest.mark.parametrize("G", ["", "1", "2", "4", "8", "16"])
def test_variable_records(oracle_mod, build_env, n, m, d, arity, G):
    """The variable-length layout (forced with MBRWT_ROWS_VAR=1; every lane
    split G) answers every row-record query like the oracle, its V / L
    accounting equals the node image's, and its export rebuilds the tree."""
    O = oracle_mod
    import torch
    from genome_graph_annotation_amd import BRWTDevice
    build_env("MBRWT_ROWS_VAR", "1")
    if G:
        build_env("MBRWT_VAR_G", G)
    rng = np.random.default_rng(n + m + len(G))
    dense = rng.random((n, m)) < d
    dense[n // 3: n // 3 + 70] = rng.random((70, m)) < 0.9  # a run of very long rows: tiles beyond the LDS budget
    t = O.OracleTree.from_dense(dense, "basic", arity)
    ex = t.export()
    dev = BRWTDevice.from_tree(ex, layout="rows")
    assert dev.layout() == "rows" and dev.rows_stats()["variable"]
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 3000), np.arange(n // 3, n // 3 + 70)]).astype(np.uint64)
    _check_all(t, dev, rows, dense)
    np.testing.assert_array_equal(_count_labels(dev, rows), dense[rows.astype(np.int64)].sum(axis=0))
    rt = torch.from_numpy(rows.view(np.int64)).cuda()
    nodes = BRWTDevice.from_tree(ex, layout="nodes")
    assert dev.count_work_device(rt) == nodes.count_work_device(rt)
    from test_gpu_files import _same_tree
    _same_tree(ex, dev.export())


@pytest.mark.parametrize("force", ["1", ""])
def test_variable_records_wide_units(oracle_mod, build_env, force):
    """Rows of ~1,230 labels (4,096 columns, arity 4, 1,024 units, d = 0.3):
    the decode's full-size per-wave budget (record chunks, owners, label stage)
    for 4 waves plus the unit table would need ~245 KB of LDS (ADVICE r04;
    the RWT table's 8,192 words bound the unit table itself to a few KB).  The budget is scaled to the workgroup's LDS;
    forced, the variable-length records answer through the global path;
    under AUTO the build declines them (a mean tile no longer fits) and the
    rows stay queryable on the other layouts."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    if force:
        build_env("MBRWT_ROWS_VAR", force)
    n, m, d = 1500, 4096, 0.3
    rng = np.random.default_rng(77)
    dense = rng.random((n, m)) < d
    t = O.OracleTree.from_dense(dense, "basic", 4)
    dev = BRWTDevice.from_tree(t.export(), layout=None)
    assert bool(force) == bool((dev.rows_stats() or {}).get("variable")), dev.rows_stats()
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 500)]).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    off_d, cols_d = dev.get_rows(rows)
    np.testing.assert_array_equal(off_d, off_o)
    np.testing.assert_array_equal(cols_d, cols_o)


def test_variable_records_ranged_async_and_errors(oracle_mod, build_env):
    """Several ranges (one record allocation each), the asynchronous call with
    its status block, capacity and range errors on the variable layout."""
    O = oracle_mod
    import torch
    from genome_graph_annotation_amd import BRWTDevice, _lib as L
    build_env("MBRWT_ROWS_RANGE", "360360")
    build_env("MBRWT_ROWS_VAR", "1")
    n, m, d = 1_100_000, 700, 0.02
    dev = BRWTDevice.synthetic(n, m, d, 8, 9, layout="rows")
    assert dev.rows_stats()["variable"]
    t = O.OracleTree.topdown(n, m, d, 8, 9)
    rows = np.concatenate([np.arange(360350, 360370), np.arange(720710, 720730), [0, n - 1],
                           np.random.default_rng(1).integers(0, n, 200_000)]).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    off_d, cols_d = dev.get_rows(rows)
    np.testing.assert_array_equal(off_d, off_o)
    np.testing.assert_array_equal(cols_d, cols_o)
    s = torch.cuda.current_stream().cuda_stream
    rt = torch.from_numpy(rows.view(np.int64)).cuda()
    ot = torch.empty(len(rows) + 1, dtype=torch.int64, device="cuda")
    ct = torch.empty(len(cols_o) + 8, dtype=torch.int32, device="cuda")
    st = torch.zeros(3, dtype=torch.int64, device="cuda")
    dev.get_rows_device_async(rt, ot, ct, st, s)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [len(cols_o), L.MBRWT_OK, 1 << L.MBRWT_OK]
    np.testing.assert_array_equal(ct[:len(cols_o)].cpu().numpy().view(np.uint32), cols_o)
    small = torch.empty(5, dtype=torch.int32, device="cuda")
    st.zero_()
    dev.get_rows_device_async(rt, ot, small, st, s)
    torch.cuda.synchronize()
    assert st.cpu().tolist()[:2] == [len(cols_o), L.MBRWT_ERR_CAPACITY]
    with pytest.raises(L.MBRWTError) as ei:
        dev.get_rows(np.array([0, n], dtype=np.uint64))
    assert ei.value.status == L.MBRWT_ERR_RANGE
    for c in (0, 3, m - 1):
        assert dev.get_column(c).tolist() == t.get_column(c)


@pytest.mark.parametrize("layout", ["rows", "nodes"])
def test_clone_concurrent_streams(oracle_mod, layout):
    """mbrwt_ctx_clone: a second query context over the same image answers
    like the oracle while the source's queries run on another stream (their
    workspaces are separate), and outlives the source (the image is freed
    with the last clone)."""
    O = oracle_mod
    import torch
    from genome_graph_annotation_amd import BRWTDevice
    n, m = 200_000, 2652
    src = BRWTDevice.synthetic(n, m, 0.003, 8, 7, layout=layout)
    cl = src.clone()
    assert cl.layout() == src.layout() and cl.num_rows() == n and cl.device_bytes() == src.device_bytes()
    t = O.OracleTree.topdown(n, m, 0.003, 8, 7)
    rng = np.random.default_rng(3)
    batches = [rng.integers(0, n, 50_000, dtype=np.uint64) for _ in range(2)]
    want = [t.get_rows(b) for b in batches]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    for j in range(2):
        rt = torch.from_numpy(batches[j].view(np.int64)).cuda()
        outs.append((rt, torch.empty(len(batches[j]) + 1, dtype=torch.int64, device="cuda"),
                     torch.empty(len(want[j][1]) + 64, dtype=torch.int32, device="cuda"),
                     torch.zeros(3, dtype=torch.int64, device="cuda")))
    torch.cuda.synchronize()
    for _ in range(8):  # interleaved on two streams, no host synchronisation
        for j, ctx in enumerate((src, cl)):
            rt, off, cols, st = outs[j]
            ctx.get_rows_device_async(rt, off, cols, st, streams[j].cuda_stream)
    torch.cuda.synchronize()
    for j in range(2):
        rt, off, cols, st = outs[j]
        assert st.cpu().tolist()[1:] == [0, 1]
        np.testing.assert_array_equal(off.cpu().numpy().view(np.uint64), want[j][0])
        np.testing.assert_array_equal(cols[:len(want[j][1])].cpu().numpy().view(np.uint32), want[j][1])
    src.close()  # the clone keeps the image
    off_d, cols_d = cl.get_rows(batches[0])
    np.testing.assert_array_equal(off_d, want[0][0])
    np.testing.assert_array_equal(cols_d, want[0][1])
    c2 = cl.clone()  # a clone of a clone shares the same image
    off_d, cols_d = c2.get_rows(batches[1])
    np.testing.assert_array_equal(cols_d, want[1][1])
    cl.close()
    off_d, cols_d = c2.get_rows(batches[1])
    np.testing.assert_array_equal(cols_d, want[1][1])
    c2.close()


def test_rows_compact_footprint(oracle_mod):
    """MBRWT_BUILD_ROWS_FOOTPRINT = MBRWT_ROWS_COMPACT: the greedy + relax
    shape's records in a smaller (or equal) image than the default's, every
    row like the oracle."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice, _lib as L
    from genome_graph_annotation_amd.brwt import build_option
    rng = np.random.default_rng(17)
    n, m = 30_000, 600
    dense = rng.random((n, m)) < 0.012
    t = O.OracleTree.from_dense(dense, "greedy", 2, 10)
    ex = t.export()
    fast = BRWTDevice.from_tree(ex, layout="rows")
    with build_option(L.MBRWT_BUILD_ROWS_FOOTPRINT, L.MBRWT_ROWS_COMPACT):
        comp = BRWTDevice.from_tree(ex, layout="rows")
    assert comp.device_bytes() <= fast.device_bytes()
    sf, sc = fast.rows_stats(), comp.rows_stats()
    assert sc["block_bytes"] / sc["rows_per_block"] <= sf["block_bytes"] / sf["rows_per_block"]
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 20_000)]).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    for d in (fast, comp):
        off_d, cols_d = d.get_rows(rows)
        np.testing.assert_array_equal(off_d, off_o)
        np.testing.assert_array_equal(cols_d, cols_o)
