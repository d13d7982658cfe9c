"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle.

Every comparison is bit-exact on the ordered CSR (ints/indices, no
tolerance).  The cases mirror the reference's own tests:
  tests/test_BRWT.cpp:152-212        all grids 1..19 x 1..19: all-zero, all-one, mixed
  tests/test_BRWT_optimizer.cpp:102-163  the same after BRWTOptimizer::relax
  experiments/run_benchmarks.py:47   C1 densities (1M x 500, arity 2)
  BASELINE.json configs[1..3]        C2 exact, C3/C4 shapes via the top-down generator
"""
import numpy as np
import pytest

from conftest import gpu_available

# the per-node images (the library default, AUTO, builds row records:
# tests/test_gpu_rows.py); a test passing layout= explicitly overrides it
pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU"),
              pytest.mark.usefixtures("nodes_layout")]


def _dev(tree):
    from genome_graph_annotation_amd import BRWTDevice
    return BRWTDevice.from_tree(tree.export())


def _check_rows(oracle_tree, dev, rows, variants=(0, 1, 2, 4, 5, 10, 17, 18, 19, 20, 24, 25, 26, 27, 28, 29, 30)):
    """Every traversal kernel (1 lane-per-row; 2/3/4 group-cooperative with
    1/2/4 children per lane; 0 the default) must
    reproduce the oracle's ordered CSR exactly."""
    from genome_graph_annotation_amd import _lib as L
    if variants is None:
        variants = _check_rows.__defaults__[0]
    from conftest import kernel_variants
    off_o, cols_o = oracle_tree.get_rows(rows)
    for v in kernel_variants(dev, variants):
        dev.set_option(L.MBRWT_OPT_KERNEL, v)
        off_d, cols_d = dev.get_rows(rows)
        np.testing.assert_array_equal(off_d, off_o)
        np.testing.assert_array_equal(cols_d, cols_o)
    dev.set_option(L.MBRWT_OPT_KERNEL, 0)
    return off_o, cols_o


def _grid(kind, n, m):
    if kind == "zero":
        return np.zeros((n, m), dtype=bool)
    if kind == "one":
        return np.ones((n, m), dtype=bool)
    i = np.arange(n)[:, None]
    j = np.arange(m)[None, :]
    return ((i + 2 * j) % 2).astype(bool)  # test_BRWT.cpp:200


@pytest.mark.parametrize("kind", ["zero", "one", "mixed"])
@pytest.mark.parametrize("build", [("basic", 2, 0), ("basic", 2, 2**64 - 1), ("greedy", 2, 0)])
def test_reference_grids(oracle_mod, kind, build):
    O = oracle_mod
    part, arity, relax = build
    for n in range(1, 20):
        for m in range(1, 20):
            dense = _grid(kind, n, m)
            t = O.OracleTree.from_dense(dense, part, arity, relax)
            d = _dev(t)
            assert d.num_rows() == n and d.num_columns() == m
            assert d.num_relations() == int(dense.sum())
            off, cols = _check_rows(t, d, np.arange(n, dtype=np.uint64))
            for i in range(n):  # the reference test compares as sets (test_BRWT.cpp:125-141)
                assert sorted(cols[off[i]:off[i + 1]].tolist()) == np.nonzero(dense[i])[0].tolist()
            ii, jj = np.meshgrid(np.arange(n), np.arange(m), indexing="ij")
            got = d.get_batch(ii.ravel(), jj.ravel())
            np.testing.assert_array_equal(got, dense.ravel())


@pytest.mark.parametrize("n,m,d,part,arity,relax", [
    (5000, 40, 0.1, "basic", 2, 0),
    (5000, 40, 0.1, "basic", 3, 0),
    (5000, 40, 0.1, "greedy", 2, 0),
    (5000, 40, 0.1, "greedy", 2, 4),
    (3000, 100, 0.05, "basic", 8, 0),
    (3000, 100, 0.05, "basic", 2, 2**64 - 1),
    (2000, 70, 0.3, "basic", 33, 0),   # MASK64 leaf parents, 64-bit masks
    (2000, 64, 0.02, "basic", 64, 0),
    (2000, 200, 0.02, "basic", 16, 0),
    (1000, 7, 1.0, "basic", 2, 0),     # dense rows
    (1000, 7, 0.0, "basic", 2, 0),     # empty matrix rows
])
def test_random_matrices(oracle_mod, n, m, d, part, arity, relax):
    O = oracle_mod
    rng = np.random.default_rng(n * 7 + m)
    dense = rng.random((n, m)) < d
    t = O.OracleTree.from_dense(dense, part, arity, relax)
    dev = _dev(t)
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 5000)]).astype(np.uint64)
    off, cols = _check_rows(t, dev, rows)
    for k in range(0, len(rows), 97):
        assert sorted(cols[off[k]:off[k + 1]].tolist()) == np.nonzero(dense[rows[k]])[0].tolist()


def test_single_column_and_empty(oracle_mod):
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice, MBRWTError
    dense = np.array([[1], [0], [1], [1]], dtype=bool)
    t = O.OracleTree.from_dense(dense)
    d = _dev(t)
    _check_rows(t, d, np.arange(4, dtype=np.uint64))
    # empty BRWT (test_BRWT.cpp:15-25): no rows, any query is out of range
    e = BRWTDevice.from_tree(O.OracleTree.from_dense(np.zeros((0, 0), dtype=bool)).export())
    assert e.num_rows() == 0 and e.num_columns() == 0
    with pytest.raises(MBRWTError):
        e.get_rows(np.array([0], dtype=np.uint64))


def test_errors_and_capacity(oracle_mod):
    O = oracle_mod
    import ctypes as C
    from genome_graph_annotation_amd import MBRWTError, _lib as L
    rng = np.random.default_rng(3)
    dense = rng.random((100, 20)) < 0.5
    t = O.OracleTree.from_dense(dense, "basic", 4)
    d = _dev(t)
    with pytest.raises(MBRWTError) as ei:
        d.get_rows(np.array([0, 100], dtype=np.uint64))
    assert ei.value.status == L.MBRWT_ERR_RANGE
    with pytest.raises(MBRWTError):
        d.get_batch([0], [20])
    # capacity retry protocol
    rows = np.arange(100, dtype=np.uint64)
    off = np.zeros(101, dtype=np.uint64)
    cols = np.zeros(5, dtype=np.uint32)
    need = C.c_uint64(0)
    st = L.lib().mbrwt_get_rows(d._h, rows.ctypes.data_as(L.u64p), 100, off.ctypes.data_as(L.u64p),
                                cols.ctypes.data_as(L.u32p), 5, C.byref(need))
    assert st == L.MBRWT_ERR_CAPACITY and need.value == int(dense.sum())
    # empty batch
    o2, c2 = d.get_rows(np.zeros(0, dtype=np.uint64))
    assert o2.tolist() == [0] and len(c2) == 0


def test_overflow_rows_take_direct_path(oracle_mod):
    """Rows with more labels than the fast path's slot take pass 2."""
    O = oracle_mod
    from genome_graph_annotation_amd import _lib as L
    rng = np.random.default_rng(5)
    dense = rng.random((3000, 300)) < 0.2  # ~60 labels per row
    t = O.OracleTree.from_dense(dense, "basic", 8)
    d = _dev(t)
    for k in (16, 32, 64, 1024):
        d.set_option(L.MBRWT_OPT_SLOT_LABELS, k)
        _check_rows(t, d, rng.integers(0, 3000, 20000).astype(np.uint64))


@pytest.mark.parametrize("density", [0.0, 0.0058333, 0.01])
def test_c1_norepl_arity2(oracle_mod, density):
    """BASELINE configs[0] (C1): 1M x 500 norepl, arity 2, mt19937 seed 42;
    queries = generate_random_ints(1000, 0, n) seed 42 (experiments/main.cpp:78-93)
    plus a 200k-row random batch."""
    O = oracle_mod
    n, m = 1_000_000, 500
    t = O.OracleTree.norepl(n, m, density, 42, "basic", 2)
    d = _dev(t)
    _check_rows(t, d, O.generate_random_ints(1000, 0, n, 42))
    _check_rows(t, d, np.random.default_rng(42).integers(0, n, 200_000).astype(np.uint64))


@pytest.mark.parametrize("layout", ["nodes", "rows"])
def test_c2_kingsford_small_exact(oracle_mod, layout):
    """BASELINE configs[1] (C2): 1M x 2,652, d=0.3%, arity 8, batch 1M --
    the reference's own generator (column-major mt19937, seed 42) and
    bottom-up builder; every row of the batch compared bit-exactly, on the
    per-node images (every kernel variant) and on the row records (the
    bench's layout)."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    n, m = 1_000_000, 2652
    t = O.OracleTree.norepl(n, m, 0.003, 42, "basic", 8)
    d = BRWTDevice.from_tree(t.export(), layout=layout)
    assert d.layout() == layout
    rows = np.random.default_rng(42).integers(0, n, 1_000_000).astype(np.uint64)
    _check_rows(t, d, rows, variants=None if layout == "nodes" else (0,))
    if layout == "rows":
        assert d.traverse_kernel() == "k_traverse_rows" and d.rows_stats()["uniform_levels"] == 3


@pytest.mark.parametrize("n,m,dens,arity", [
    (2_000_000, 2652, 0.003, 8),   # Kingsford shape, reduced rows
    (300_000, 3173, 0.038, 8),     # RefSeq shape, reduced rows
    (50_000, 4000, 0.003, 8),      # > kLdsNodes internal records: fast kernel, global record fallback
    (100_000, 1, 0.3, 2),          # root is a leaf
    (100_000, 2, 0.5, 2),
    (200_000, 500, 0.01, 2),
    (200_000, 1000, 0.02, 3),
    (100_000, 700, 0.05, 12),      # MASK16 leaf parents
])
def test_synthetic_matches_oracle(oracle_mod, n, m, dens, arity):
    """The device generator and the oracle's independent implementation of
    the same spec produce the same BRWT (same answers on every sampled row)."""
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    t = O.OracleTree.topdown(n, m, dens, arity, 42)
    d = BRWTDevice.synthetic(n, m, dens, arity, 42)
    assert d.num_relations() == t.num_relations()
    assert d.num_rows() == n and d.num_columns() == m
    rows = np.random.default_rng(1).integers(0, n, 300_000).astype(np.uint64)
    _check_rows(t, d, rows)


def test_device_api_and_accounting(oracle_mod):
    import torch
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice
    n, m = 500_000, 2652
    t = O.OracleTree.topdown(n, m, 0.003, 8, 7)
    d = BRWTDevice.synthetic(n, m, 0.003, 8, 7)
    rows = np.random.default_rng(2).integers(0, n, 100_000).astype(np.uint64)
    off_o, cols_o, vis = t.get_rows(rows, with_visits=True)
    rt = torch.from_numpy(rows.view(np.int64)).cuda()
    ot = torch.empty(len(rows) + 1, dtype=torch.int64, device="cuda")
    ct = torch.empty(len(cols_o) + 10, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    got = d.get_rows_device(rt, ot, ct, s.cuda_stream)
    torch.cuda.synchronize()
    assert got == len(cols_o)
    np.testing.assert_array_equal(ot.cpu().numpy().view(np.uint64), off_o)
    np.testing.assert_array_equal(ct[:got].cpu().numpy().view(np.uint32), cols_o)
    from genome_graph_annotation_amd import _lib as L
    from conftest import kernel_variants
    for variant in kernel_variants(d, (0, 1, 2, 4)):
        d.set_option(L.MBRWT_OPT_KERNEL, variant)
        # V and L accounting used by the roofline (DESIGN.md "Measurement")
        v, lab = d.count_work_device(rt, s.cuda_stream)
        assert v == int(vis.sum()) and lab == len(cols_o)
        # fused count_labels (annotate_static.cpp:149-162)
        cnt = torch.empty(m, dtype=torch.int64, device="cuda")
        d.count_labels_device(rt, cnt, s.cuda_stream)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(cnt.cpu().numpy(), np.bincount(cols_o, minlength=m))


# ---- BRWT::get_column (BRWT.cpp:55-85), §8f row 4 ------------------------------

def _check_columns(oracle_tree, dev, cols):
    for j in cols:
        want = np.asarray(oracle_tree.get_column(int(j)), dtype=np.uint64)
        got = dev.get_column(int(j))
        np.testing.assert_array_equal(got, want, err_msg=f"column {j}")


@pytest.mark.parametrize("kind", ["zero", "one", "mixed"])
@pytest.mark.parametrize("build", [("basic", 2, 0), ("basic", 2, 2**64 - 1), ("greedy", 2, 0)])
def test_get_column_reference_grids(oracle_mod, kind, build):
    """test_BRWT.cpp:105-123 over the 1..19 x 1..19 grids: every column, the
    ascending row list of the oracle (the dense matrix pins it too)."""
    O = oracle_mod
    part, arity, relax = build
    for n in range(1, 20, 3):
        for m in range(1, 20, 2):
            dense = _grid(kind, n, m)
            t = O.OracleTree.from_dense(dense, part, arity, relax)
            d = _dev(t)
            for j in range(m):
                got = d.get_column(j)
                np.testing.assert_array_equal(got, np.nonzero(dense[:, j])[0].astype(np.uint64))
            _check_columns(t, d, range(m))


@pytest.mark.parametrize("n,m,dens,part,arity", [
    (5000, 40, 0.1, "greedy", 2),
    (3000, 100, 0.05, "basic", 8),
    (2000, 70, 0.3, "basic", 33),      # MASK64 leaf parents
    (2000, 200, 0.02, "basic", 16),    # MASK16
    (4000, 9, 0.5, "basic", 8),        # leaves directly under a PLANE node (8 + 1 columns)
    (70_000, 5, 0.9, "basic", 2),      # long dense columns, several lift levels
])
def test_get_column_random(oracle_mod, n, m, dens, part, arity):
    O = oracle_mod
    rng = np.random.default_rng(n + m)
    dense = rng.random((n, m)) < dens
    t = O.OracleTree.from_dense(dense, part, arity)
    d = _dev(t)
    for j in range(m):
        np.testing.assert_array_equal(d.get_column(j), np.nonzero(dense[:, j])[0].astype(np.uint64))


def test_get_column_synthetic_and_errors(oracle_mod):
    """Kingsford-shaped synthetic tree (root folded) and the capacity/range
    protocol of mbrwt_get_column[_device]."""
    import torch
    O = oracle_mod
    from genome_graph_annotation_amd import BRWTDevice, MBRWTError, _lib as L
    n, m = 2_000_000, 2652
    t = O.OracleTree.topdown(n, m, 0.003, 8, 42)
    d = BRWTDevice.synthetic(n, m, 0.003, 8, 42)
    cols = np.random.default_rng(4).integers(0, m, 48).tolist() + [0, m - 1]
    _check_columns(t, d, cols)
    with pytest.raises(MBRWTError) as ei:
        d.get_column(m)
    assert ei.value.status == L.MBRWT_ERR_RANGE
    want = np.asarray(t.get_column(7), dtype=np.uint64)
    small = torch.empty(max(0, len(want) - 1), dtype=torch.int64, device="cuda")
    with pytest.raises(MBRWTError) as ei:
        d.get_column_device(7, small)
    assert ei.value.status == L.MBRWT_ERR_CAPACITY and ei.value.needed == len(want)
    big = torch.empty(len(want) + 3, dtype=torch.int64, device="cuda")
    got = d.get_column_device(7, big, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert got == len(want)
    np.testing.assert_array_equal(big[:got].cpu().numpy().view(np.uint64), want)


# ---- KIND_PACK layout (mbrwt_internal.hpp) vs the plain PLANE + MASK8 layout ----

def _with_env(name, value, fn):
    """fn() under the build option that replaced the r04 switch `name`."""
    from conftest import with_build
    return with_build(name, value, fn)


@pytest.fixture
def no_packt(build_env):
    """The PACK / PACK2 layout tests measure those layouts: no KIND_PACKT."""
    build_env("MBRWT_PACKT", "0")


def _agree(oracle_tree, devs, rows, cols, m):
    import torch
    off_o, cols_o, vis = oracle_tree.get_rows(rows, with_visits=True)
    for d in devs:
        _check_rows(oracle_tree, d, rows)
        for j in cols:
            np.testing.assert_array_equal(d.get_column(int(j)), np.asarray(oracle_tree.get_column(int(j)), dtype=np.uint64))
        rt = torch.from_numpy(rows.view(np.int64)).cuda()
        v, lab = d.count_work_device(rt, torch.cuda.current_stream().cuda_stream)
        assert v == int(vis.sum()) and lab == len(cols_o)
        ii = rows[:2000]
        jj = np.random.default_rng(3).integers(0, m, len(ii)).astype(np.uint64)
        want = np.array([oracle_tree.get(int(a), int(b)) for a, b in zip(ii, jj)])
        np.testing.assert_array_equal(d.get_batch(ii, jj), want)


def test_pack_layout_with_spills(oracle_mod, no_packt):
    """A tree whose PACK node has a few blocks with > 48 masks (spill lists):
    packed and unpacked images answer like the oracle (rows, columns, get,
    V/L accounting)."""
    O = oracle_mod
    rng = np.random.default_rng(11)
    n, m = 4000, 64
    dense = rng.random((n, m)) < 0.01
    dense[1000:1040] = True  # a run of dense rows: its PACK blocks spill
    t = O.OracleTree.from_dense(dense, "basic", 8)
    packed = _dev(t)
    plain = _with_env("MBRWT_PACK", "0", lambda: _dev(t))
    assert packed.traverse_kernel() == plain.traverse_kernel() == "k_traverse_fast2"
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 20000)]).astype(np.uint64)
    _agree(t, [packed, plain], rows, range(m), m)


@pytest.mark.parametrize("fold", ["1", "0"])
def test_pack_layout_synthetic(oracle_mod, no_packt, fold):
    """Synthetic Kingsford-shaped trees with and without PACK nodes (and with
    and without root folding) agree with the oracle."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    n, m = 400_000, 2652
    t = O.OracleTree.topdown(n, m, 0.003, 8, 5)

    def mk():
        return BRWTDevice.synthetic(n, m, 0.003, 8, 5)
    packed = _with_env("MBRWT_FOLD_ROOT", fold, mk)
    plain = _with_env("MBRWT_FOLD_ROOT", fold, lambda: _with_env("MBRWT_PACK", "0", mk))
    assert packed.device_bytes() != plain.device_bytes()
    rows = np.random.default_rng(9).integers(0, n, 100_000).astype(np.uint64)
    _agree(t, [packed, plain], rows, np.random.default_rng(2).integers(0, m, 16), m)


# ---- KIND_PACK2 layout: a node's whole 3-level subtree inline per position ----

def test_pack2_layout_with_spills(oracle_mod, no_packt):
    """Arity-4 tree (256 -> 64 -> 16 -> 4 -> root, folded): the 4 nodes under
    the root become KIND_PACK2; a run of dense rows makes a few of their
    blocks spill.  PACK2, PACK-only and plain images answer like the oracle
    (rows under every kernel, columns, get, V/L accounting)."""
    O = oracle_mod
    rng = np.random.default_rng(12)
    n, m = 4000, 256
    dense = rng.random((n, m)) < 0.004
    dense[2000:2024] = True
    t = O.OracleTree.from_dense(dense, "basic", 4)
    p2 = _dev(t)
    p1 = _with_env("MBRWT_PACK2", "0", lambda: _dev(t))
    plain = _with_env("MBRWT_PACK", "0", lambda: _dev(t))
    assert p2.traverse_kernel() == "k_traverse_p2w"  # the root's children are all PACK2
    assert p1.traverse_kernel() == plain.traverse_kernel() == "k_traverse_fast2"
    # (the dense run makes PACK decline here: > 1 block in 20 would spill)
    assert p2.device_bytes() not in (p1.device_bytes(), plain.device_bytes())
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 20000)]).astype(np.uint64)
    _agree(t, [p2, p1, plain], rows, range(m), m)


def test_pack2_records_longer_than_a_block(oracle_mod, no_packt):
    """Arity 8, 2048 columns (2048 -> 256 -> 32 -> 4 -> root): a fully set row
    gives a 73-byte record (1 + 8 + 64 masks), longer than a block: the host
    builder declines PACK2 for those nodes (mbrwt_internal.hpp) and the
    results stay the oracle's."""
    O = oracle_mod
    rng = np.random.default_rng(13)
    n, m = 3000, 2048
    dense = rng.random((n, m)) < 0.0005
    dense[[5, 1500, 1501]] = True
    t = O.OracleTree.from_dense(dense, "basic", 8)
    p2 = _dev(t)
    assert p2.traverse_kernel() == "k_traverse_fast2"
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 5000)]).astype(np.uint64)
    _agree(t, [p2], rows, [0, 7, 8, 511, 512, 2047], m)


@pytest.mark.parametrize("fold", ["1", "0"])
def test_pack2_layout_synthetic(oracle_mod, no_packt, fold):
    """Synthetic Kingsford-shaped trees: the generator's PACK2 images (default)
    agree with the oracle, as do PACK-only images."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    n, m = 400_000, 2652
    t = O.OracleTree.topdown(n, m, 0.003, 8, 6)

    def mk():
        return BRWTDevice.synthetic(n, m, 0.003, 8, 6)
    p2 = _with_env("MBRWT_FOLD_ROOT", fold, mk)
    p1 = _with_env("MBRWT_FOLD_ROOT", fold, lambda: _with_env("MBRWT_PACK2", "0", mk))
    assert p2.device_bytes() != p1.device_bytes()
    # folded: the super-root's children are the PACK2 nodes (k_traverse_p2w);
    # unfolded: the super-root's child is the PLANE root (two stack frames: the
    # general kernel)
    if fold == "1":
        assert p2.traverse_kernel() == "k_traverse_p2w"
    rows = np.random.default_rng(10).integers(0, n, 100_000).astype(np.uint64)
    _agree(t, [p2, p1], rows, np.random.default_rng(4).integers(0, m, 16), m)


def test_pack2_dense_subtrees_take_a_short_span(oracle_mod, no_packt):
    """d = 4 %: ~26 record bytes per position, so the host builder picks a
    span of 2 or 1 positions per block (mbrwt_internal.hpp); results as the
    oracle's under every kernel."""
    O = oracle_mod
    rng = np.random.default_rng(14)
    n, m = 3000, 2048
    dense = rng.random((n, m)) < 0.04
    t = O.OracleTree.from_dense(dense, "basic", 8)
    p2 = _dev(t)
    p1 = _with_env("MBRWT_PACK2", "0", lambda: _dev(t))
    assert p2.traverse_kernel() == "k_traverse_p2w"
    assert p2.device_bytes() != p1.device_bytes()
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 5000)]).astype(np.uint64)
    _agree(t, [p2, p1], rows, [0, 9, 100, 1023, 2047], m)


def test_pack2_refseq_shape_synthetic(oracle_mod, no_packt):
    """RefSeq shape (3,173 columns, d = 3.8 %): the generator's span-2 PACK2
    images agree with the oracle's independent implementation of the spec."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    n, m = 200_000, 3173
    t = O.OracleTree.topdown(n, m, 0.038, 8, 8)
    p2 = BRWTDevice.synthetic(n, m, 0.038, 8, 8)
    p1 = _with_env("MBRWT_PACK2", "0", lambda: BRWTDevice.synthetic(n, m, 0.038, 8, 8))
    assert p2.traverse_kernel() == "k_traverse_p2w"
    assert p2.device_bytes() != p1.device_bytes()
    rows = np.random.default_rng(11).integers(0, n, 20_000).astype(np.uint64)
    _agree(t, [p2, p1], rows, np.random.default_rng(5).integers(0, m, 6), m)


# ---- device builder (mbrwt_create_from_columns): BRWTBottomUpBuilder::build ----

def _oracle_from_words(O, words, n, m, arity):
    return O.OracleTree(O.lib().oracle_build_from_columns(O._p64(words), n, m, 0, arity, 0))


@pytest.mark.parametrize("n,m,d,arity", [(1, 1, 0.5, 2), (64, 3, 0.5, 2), (1000, 37, 0.05, 2), (5000, 300, 0.01, 8),
                                         (3001, 100, 0.2, 3), (777, 130, 0.03, 64), (4096, 513, 0.004, 8)])
def test_device_builder_matches_reference_builder(oracle_mod, n, m, d, arity):
    """The device-built BRWT is the reference builder's tree: the same image
    as the oracle's tree exported through mbrwt_create (byte count) and the
    same answers to every query."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    words = O.generate_columns(n, m, d, seed=n + m)
    W = (n + 63) // 64
    t = _oracle_from_words(O, words, n, m, arity)
    built = BRWTDevice.from_columns(words[: m * W].reshape(m, W), n, arity)
    ref = BRWTDevice.from_tree(t.export())
    assert built.device_bytes() == ref.device_bytes()
    assert built.num_relations() == t.num_relations() and built.num_nodes() == ref.num_nodes()
    rows = np.concatenate([np.arange(n), np.random.default_rng(1).integers(0, n, 3000)]).astype(np.uint64)
    _agree(t, [built], rows, np.unique(np.linspace(0, m - 1, 12).astype(int)), m)


def test_device_builder_edge_cases(oracle_mod):
    from genome_graph_annotation_amd import BRWTDevice, _lib as L
    empty = BRWTDevice.from_columns([], 10, 2)  # no columns: BRWT() (BRWT_builders.cpp:122-123)
    assert empty.num_columns() == 0 and empty.num_rows() == 0
    # garbage past num_rows is ignored
    col = np.array([0xFFFFFFFFFFFFFFFF], dtype=np.uint64)
    one = BRWTDevice.from_columns([col], 10, 2)
    assert one.num_relations() == 10
    off, cols = one.get_rows(np.arange(10, dtype=np.uint64))
    assert list(off) == list(range(11)) and set(cols.tolist()) == {0}
    with pytest.raises(L.MBRWTError):
        BRWTDevice.from_columns([col], 10, 1)  # arity < 2


def test_device_builder_c2_shape(oracle_mod):
    """BASELINE configs[1] shape from the reference's own column generator
    (mt19937, data_generation.cpp:20-29): 1 M x 2,652, d = 0.3 %, arity 8."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    n, m = 1_000_000, 2652
    words = O.generate_columns(n, m, 0.003, seed=42)
    W = (n + 63) // 64
    t = _oracle_from_words(O, words, n, m, 8)
    built = BRWTDevice.from_columns(words.reshape(m, W), n, 8)
    assert built.device_bytes() == BRWTDevice.from_tree(t.export()).device_bytes()
    rows = np.random.default_rng(2).integers(0, n, 200_000).astype(np.uint64)
    _check_rows(t, built, rows, variants=(0,))


@pytest.mark.parametrize("m", [9, 17, 65, 129])
def test_device_builder_pass_through_nodes(oracle_mod, m):
    """Column counts that leave a single node in a group on several levels
    (pass-through of internal nodes, BRWT_builders.cpp:75-77), arity 2."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    n = 3000
    words = O.generate_columns(n, m, 0.05, seed=m)
    W = (n + 63) // 64
    t = _oracle_from_words(O, words, n, m, 2)
    built = BRWTDevice.from_columns(words[: m * W].reshape(m, W), n, 2)
    assert built.device_bytes() == BRWTDevice.from_tree(t.export()).device_bytes()
    _check_rows(t, built, np.arange(n, dtype=np.uint64), variants=(0,))


# ---- binary_grouping_greedy on the device (partitionings.cpp:148-196) ----

def _same_tree(a, b):
    for k in ("num_children", "first_child", "leaf_column"):
        np.testing.assert_array_equal(np.asarray(a[k]), np.asarray(b[k]), err_msg=k)


@pytest.mark.parametrize("n,m,d,relax", [
    (3000, 100, 0.05, 0), (3000, 100, 0.05, 10), (5000, 257, 0.02, 0), (20000, 64, 0.1, 10),
    (2000, 40, 0.0, 0),             # all-zero columns: every similarity ties
    (2_500_000, 24, 0.001, 10),     # 1e6 < rows <= 1e7: the Bernoulli row sample
    (12_000_000, 12, 0.0005, 0),    # rows > 1e7: the uniform row sample
])
def test_device_greedy_builder_matches_reference(oracle_mod, n, m, d, relax):
    """mbrwt_create_from_columns[_relaxed] with MBRWT_PARTITIONER_GREEDY builds
    the oracle's greedy (+ relax) tree: the same tree (exported shape), the same
    image bytes, the same answers."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    words = O.generate_columns(n, m, d, seed=n + m + 7)
    W = (n + 63) // 64
    t = O.OracleTree(O.lib().oracle_build_from_columns(O._p64(words), n, m, 1, 2, relax))
    built = BRWTDevice.from_columns(words[: m * W].reshape(m, W), n, 2, relax_max_arity=relax, partitioner="greedy")
    ref = BRWTDevice.from_tree(t.export())
    _same_tree(built.export(), t.export())
    assert built.device_bytes() == ref.device_bytes()
    rows = np.random.default_rng(3).integers(0, n, 20000).astype(np.uint64)
    _check_rows(t, built, rows, variants=(0,))


def test_device_greedy_builder_c2_production_shape(oracle_mod):
    """The reference's production build (greedy + relax 10,
    scripts/kingsford/convert.sh:24) of the C2 columns (1 M x 2,652, d = 0.3 %,
    the reference's own mt19937 generator) on the device: the oracle's tree."""
    import time
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    n, m = 1_000_000, 2652
    words = O.generate_columns(n, m, 0.003, seed=42)
    W = (n + 63) // 64
    t0 = time.time()
    built = BRWTDevice.from_columns(words.reshape(m, W), n, 2, relax_max_arity=10, partitioner="greedy")
    dev_s = time.time() - t0
    t0 = time.time()
    t = O.OracleTree(O.lib().oracle_build_from_columns(O._p64(words), n, m, 1, 2, 10))
    print(f"greedy + relax 10 of C2: device {dev_s:.2f} s, oracle {time.time() - t0:.1f} s")
    _same_tree(built.export(), t.export())
    rows = np.random.default_rng(4).integers(0, n, 100_000).astype(np.uint64)
    _check_rows(t, built, rows, variants=(0,))


# ---- BRWTOptimizer::relax on the device ----

def _oracle_from_words_relaxed(O, words, n, m, arity, relax):
    return O.OracleTree(O.lib().oracle_build_from_columns(O._p64(words), n, m, 0, arity, relax))


@pytest.mark.parametrize("n,m,d,arity,relax", [(3000, 100, 0.05, 2, 2**64 - 1), (3000, 100, 0.05, 2, 4),
                                               (5000, 300, 0.01, 2, 8), (2000, 129, 0.3, 2, 10),
                                               (4096, 513, 0.004, 3, 16), (1000, 37, 0.05, 2, 2)])
def test_device_relax_matches_reference_relax(oracle_mod, n, m, d, arity, relax):
    """Builder + relax on the device (mbrwt_create_from_columns_relaxed) and
    relax of an exported unrelaxed tree (mbrwt_create_relaxed) both give the
    oracle's relaxed tree (BRWT_builders.cpp:166-297): the same node count and
    image bytes as the oracle's relaxed tree through mbrwt_create, and the
    same answers to every query."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    words = O.generate_columns(n, m, d, seed=n + m + 1)
    W = (n + 63) // 64
    cols = words[: m * W].reshape(m, W)
    t = _oracle_from_words_relaxed(O, words, n, m, arity, relax)
    plain = _oracle_from_words(O, words, n, m, arity)
    ref = BRWTDevice.from_tree(t.export())
    built = BRWTDevice.from_columns(cols, n, arity, relax_max_arity=relax)
    from_desc = BRWTDevice.from_tree(plain.export(), relax_max_arity=relax)
    for dev in (built, from_desc):
        assert dev.num_nodes() == ref.num_nodes() and dev.device_bytes() == ref.device_bytes()
        assert dev.num_relations() == t.num_relations()
    if relax > 2:
        assert ref.num_nodes() < BRWTDevice.from_tree(plain.export()).num_nodes()  # relax pruned something
    rows = np.concatenate([np.arange(n), np.random.default_rng(1).integers(0, n, 2000)]).astype(np.uint64)
    _agree(t, [built, from_desc], rows, np.unique(np.linspace(0, m - 1, 8).astype(int)), m)


@pytest.mark.parametrize("kind", ["zero", "one", "mixed"])
def test_device_relax_reference_grids(oracle_mod, kind):
    """test_BRWT_optimizer.cpp:102-163: every grid 1..19 x 1..19, arity 2,
    relaxed with max arity 2^64-1, through mbrwt_create_relaxed."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    for n in range(1, 20):
        for m in range(1, 20):
            dense = _grid(kind, n, m)
            t = O.OracleTree.from_dense(dense, "basic", 2, 2**64 - 1)
            plain = O.OracleTree.from_dense(dense, "basic", 2, 0)
            dev = BRWTDevice.from_tree(plain.export(), relax_max_arity=2**64 - 1)
            assert dev.num_nodes() == BRWTDevice.from_tree(t.export()).num_nodes()
            off, cols = _check_rows(t, dev, np.arange(n, dtype=np.uint64), variants=(0,))
            for i in range(n):
                assert sorted(cols[off[i]:off[i + 1]].tolist()) == np.nonzero(dense[i])[0].tolist()


def test_pack_ids_kernels_match_the_wire_format():
    """mbrwt_pack_ids_device / mbrwt_unpack_ids_device (the all-gatherv's wire
    format) against dist.py's CPU reference implementation."""
    import torch
    from genome_graph_annotation_amd.dist import _pack, _unpack, _words
    rng = np.random.default_rng(6)
    for bits in (1, 5, 12, 16, 23, 32):
        for n in (1, 31, 32, 33, 100_003):
            v = rng.integers(0, 1 << bits, n, dtype=np.uint64).astype(np.uint32)
            cpu_words = torch.zeros(_words(n, bits), dtype=torch.int32)
            _pack(torch.from_numpy(v.view(np.int32)), n, bits, cpu_words)
            g = torch.from_numpy(v.view(np.int32)).cuda()
            gw = torch.zeros(_words(n, bits) + 1, dtype=torch.int32, device="cuda")
            _pack(g, n, bits, gw)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(gw[: _words(n, bits)].cpu().numpy(), cpu_words.numpy())
            out = torch.empty(n, dtype=torch.int32, device="cuda")
            _unpack(gw, n, bits, out)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), v)


# ---- batched get_labels(indices, presence_ratio): the classify consumer (§8f row 2) ----

def _ref_get_labels(off_o, cols_o, read_offsets, m, ratio):
    """annotate_static.cpp:71-94 over the oracle's rows (std::ceil in double)."""
    import math
    out_off, out = [0], []
    for r in range(len(read_offsets) - 1):
        a, b = int(read_offsets[r]), int(read_offsets[r + 1])
        cnt = np.bincount(cols_o[off_o[a]:off_o[b]], minlength=m)
        thr = 1 if ratio == 0 else math.ceil((b - a) * ratio)
        labs = np.nonzero((cnt > 0) & (cnt >= thr))[0]
        out.extend(labs.tolist())
        out_off.append(len(out))
    return np.array(out_off, dtype=np.uint64), np.array(out, dtype=np.uint32)


@pytest.mark.parametrize("ratio", [0.0, 0.1, 0.5, 1.0])
def test_get_labels_batch_matches_reference_semantics(oracle_mod, ratio):
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    n, m = 200_000, 2652
    t = O.OracleTree.topdown(n, m, 0.003, 8, 21)
    d = BRWTDevice.synthetic(n, m, 0.003, 8, 21)
    rng = np.random.default_rng(7)
    lens = rng.integers(0, 60, 3000)  # reads of 0..59 k-mer rows, some empty
    read_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    # a read's k-mers hit neighbouring rows often: draw around a per-read anchor
    anchors = rng.integers(0, n - 100, len(lens))
    rows = np.concatenate([a + rng.integers(0, 100, k) for a, k in zip(anchors, lens)]).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    want_off, want = _ref_get_labels(off_o, cols_o, read_off, m, ratio)
    got_off, got = d.get_labels_batch(rows, read_off, ratio)
    np.testing.assert_array_equal(got_off, want_off)
    np.testing.assert_array_equal(got, want)


def test_get_labels_batch_errors(oracle_mod):
    from genome_graph_annotation_amd import BRWTDevice, _lib as L
    d = BRWTDevice.synthetic(1000, 100, 0.05, 8, 3)
    rows = np.arange(10, dtype=np.uint64)
    with pytest.raises(L.MBRWTError):
        d.get_labels_batch(rows, np.array([0, 10], dtype=np.uint64), 1.5)  # an assert in the reference
    with pytest.raises(L.MBRWTError):
        d.get_labels_batch(np.array([5000], dtype=np.uint64), np.array([0, 1], dtype=np.uint64), 0.0)  # row range
    off, labs = d.get_labels_batch(rows, np.array([0, 0, 10], dtype=np.uint64), 0.0)  # an empty read
    assert off[0] == 0 and off[1] == 0 and off[2] == len(labs)
    for bad in ([0, 11], [1, 10], [0, 6, 4, 10], [0, 5, 9]):  # past n_rows, not from 0, descending, short
        with pytest.raises(L.MBRWTError) as e:
            d.get_labels_batch(rows, np.array(bad, dtype=np.uint64), 0.0)
        assert e.value.status == L.MBRWT_ERR_INVALID
    off, labs = d.get_labels_batch(np.zeros(0, dtype=np.uint64), np.array([0], dtype=np.uint64), 0.5)  # no reads
    assert off.tolist() == [0] and labs.size == 0
    none = np.zeros(0, dtype=np.uint64)
    off, labs = d.get_labels_batch(none, np.array([0, 0, 0], dtype=np.uint64), 0.0)  # reads without rows
    assert off.tolist() == [0, 0, 0] and labs.size == 0
    off, labs, cnts = d.get_top_labels_batch(none, np.array([0, 0], dtype=np.uint64), 5)
    assert off.tolist() == [0, 0] and labs.size == 0 and cnts.size == 0
    with pytest.raises(L.MBRWTError) as e:  # zero reads but rows: the one offset cannot be 0 and n_rows
        d.get_labels_batch(rows, np.array([0], dtype=np.uint64), 0.0)
    assert e.value.status == L.MBRWT_ERR_INVALID


def test_get_labels_batch_device_matches_host(oracle_mod):
    """The device-buffer form (torch tensors as plumbing, capacity protocol)
    returns what the host-buffer form returns."""
    import torch
    from genome_graph_annotation_amd import BRWTDevice, _lib as L
    n, m = 100_000, 700
    d = BRWTDevice.synthetic(n, m, 0.01, 8, 5)
    rng = np.random.default_rng(9)
    lens = rng.integers(1, 40, 2000)
    read_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    rows = rng.integers(0, n, int(read_off[-1])).astype(np.uint64)
    want_off, want = d.get_labels_batch(rows, read_off, 0.25)
    rt = torch.from_numpy(rows.view(np.int64)).cuda()
    ot = torch.from_numpy(read_off.view(np.int64)).cuda()
    lo = torch.empty(len(read_off), dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    small = torch.empty(1, dtype=torch.int32, device="cuda")
    with pytest.raises(L.MBRWTError) as e:
        d.get_labels_batch_device(rt, ot, 0.25, lo, small, s)
    assert e.value.needed == len(want)
    lt = torch.empty(e.value.needed, dtype=torch.int32, device="cuda")
    got = d.get_labels_batch_device(rt, ot, 0.25, lo, lt, s)
    torch.cuda.synchronize()
    assert got == len(want)
    np.testing.assert_array_equal(lo.cpu().numpy().view(np.uint64), want_off)
    np.testing.assert_array_equal(lt.cpu().numpy().view(np.uint32), want)


# ---- batched get_top_labels(indices, num_top): classify --count-labels (§8f row 2) ----

def _ref_top_labels(off_o, cols_o, read_offsets, m, num_top):
    """annotate.cpp:57-83 over the oracle's rows; equal counts put in ascending
    label order (the reference's std::sort leaves them unspecified)."""
    out_off, labs, cnts = [0], [], []
    for r in range(len(read_offsets) - 1):
        a, b = int(read_offsets[r]), int(read_offsets[r + 1])
        cnt = np.bincount(cols_o[off_o[a]:off_o[b]], minlength=m)
        nz = np.nonzero(cnt)[0]
        order = nz[np.lexsort((nz, -cnt[nz].astype(np.int64)))][:num_top]
        labs.extend(order.tolist())
        cnts.extend(cnt[order].tolist())
        out_off.append(len(labs))
    return (np.array(out_off, dtype=np.uint64), np.array(labs, dtype=np.uint32), np.array(cnts, dtype=np.uint64))


# density 0.2 at m = 2652: most reads hold > 1024 distinct labels (the in-place
# whole-histogram sort); the others fit the compact buffer
@pytest.mark.parametrize("m,num_top,dens", [(2652, 2**64 - 1, 0.003), (2652, 5, 0.003), (2652, 1, 0.003),
                                            (2652, 0, 0.003), (8192, 20, 0.003), (3, 2, 0.3),
                                            (2652, 2**64 - 1, 0.2), (2652, 50, 0.2)])
def test_get_top_labels_batch_matches_reference_semantics(oracle_mod, m, num_top, dens):
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    n = 100_000 if dens < 0.1 else 5_000
    t = O.OracleTree.topdown(n, m, dens, 8, 31)
    d = BRWTDevice.synthetic(n, m, dens, 8, 31)
    rng = np.random.default_rng(11)
    lens = rng.integers(0, 80, 1500 if dens < 0.1 else 200)
    read_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    anchors = rng.integers(0, n - 50, len(lens))
    rows = np.concatenate([a + rng.integers(0, 50, k) for a, k in zip(anchors, lens)]).astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    want_off, want_l, want_c = _ref_top_labels(off_o, cols_o, read_off, m, min(num_top, m + 1))
    got_off, got_l, got_c = d.get_top_labels_batch(rows, read_off, num_top)
    np.testing.assert_array_equal(got_off, want_off)
    np.testing.assert_array_equal(got_l, want_l)
    np.testing.assert_array_equal(got_c, want_c)


def test_get_top_labels_batch_errors_and_device_form(oracle_mod):
    import torch
    from genome_graph_annotation_amd import BRWTDevice, _lib as L
    big = BRWTDevice.synthetic(1000, 8193, 0.001, 8, 3)
    with pytest.raises(L.MBRWTError) as e:
        big.get_top_labels_batch(np.arange(4, dtype=np.uint64), np.array([0, 4], dtype=np.uint64), 3)
    assert e.value.status == L.MBRWT_ERR_UNSUPPORTED
    d = BRWTDevice.synthetic(50_000, 700, 0.01, 8, 5)
    rows = np.arange(10, dtype=np.uint64)
    for bad in ([0, 11], [1, 10], [0, 6, 4, 10]):
        with pytest.raises(L.MBRWTError) as e:
            d.get_top_labels_batch(rows, np.array(bad, dtype=np.uint64), 3)
        assert e.value.status == L.MBRWT_ERR_INVALID
    rng = np.random.default_rng(2)
    lens = rng.integers(1, 40, 1000)
    read_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    rows = rng.integers(0, 50_000, int(read_off[-1])).astype(np.uint64)
    want = d.get_top_labels_batch(rows, read_off, 7)
    rt = torch.from_numpy(rows.view(np.int64)).cuda()
    ot = torch.from_numpy(read_off.view(np.int64)).cuda()
    lo = torch.empty(len(read_off), dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    with pytest.raises(L.MBRWTError) as e:
        d.get_top_labels_batch_device(rt, ot, 7, lo, None, None, s)
    n = e.value.needed
    assert n == len(want[1])
    lt = torch.empty(n, dtype=torch.int32, device="cuda")
    ct = torch.empty(n, dtype=torch.int64, device="cuda")
    assert d.get_top_labels_batch_device(rt, ot, 7, lo, lt, ct, s) == n
    torch.cuda.synchronize()
    np.testing.assert_array_equal(lo.cpu().numpy().view(np.uint64), want[0])
    np.testing.assert_array_equal(lt.cpu().numpy().view(np.uint32), want[1])
    np.testing.assert_array_equal(ct.cpu().numpy().view(np.uint64), want[2])


@pytest.mark.parametrize("relax", [2, 4, 2**64 - 1])
def test_device_relax_of_greedy_trees(oracle_mod, relax):
    """mbrwt_create_relaxed on an exported greedy-partitioned tree (non-contiguous
    column groups) against the oracle's relax of the same tree
    (BRWT_builders.cpp:166-297 keeps the column arrangement): same node count,
    same ordered CSR."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    rng = np.random.default_rng(17 + relax % 97)
    n, m = 3000, 60
    dense = rng.random((n, m)) < 0.08
    t = O.OracleTree.from_dense(dense, "greedy", 2, relax)
    plain = O.OracleTree.from_dense(dense, "greedy", 2, 0)
    dev = BRWTDevice.from_tree(plain.export(), relax_max_arity=relax)
    assert dev.num_nodes() == BRWTDevice.from_tree(t.export()).num_nodes()
    rows = np.arange(n, dtype=np.uint64)
    off, cols = _check_rows(t, dev, rows, variants=(0,))
    for k in range(0, n, 37):
        assert sorted(cols[off[k]:off[k + 1]].tolist()) == np.nonzero(dense[k])[0].tolist()


def test_device_calls_on_two_streams(oracle_mod):
    """Workspaces are ordered across the callers' streams (include/mbrwt.h
    "Threading"): a get_rows_device queued on stream A and one issued right
    after on stream B (no host sync in between) both match the oracle."""
    import torch
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    n, m = 300_000, 2652
    dev = BRWTDevice.synthetic(n, m, 0.003, 8, 11)
    ref = O.OracleTree.topdown(n, m, 0.003, 8, 11)
    rng = np.random.default_rng(5)
    batches = [rng.integers(0, n, k).astype(np.uint64) for k in (400_000, 50_000)]
    want = [ref.get_rows(b) for b in batches]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    for b, w, s in zip(batches, want, streams):
        with torch.cuda.stream(s):
            rt = torch.from_numpy(b.view(np.int64)).to("cuda", non_blocking=False)
            ot = torch.empty(len(b) + 1, dtype=torch.int64, device="cuda")
            ct = torch.empty(len(w[1]) + 16, dtype=torch.int32, device="cuda")
            s.synchronize()
            got = dev.get_rows_device(rt, ot, ct, s.cuda_stream)
            outs.append((got, ot, ct, rt))
    torch.cuda.synchronize()
    for (got, ot, ct, _), (off_o, cols_o) in zip(outs, want):
        assert got == len(cols_o)
        np.testing.assert_array_equal(ot.cpu().numpy().view(np.uint64), off_o)
        np.testing.assert_array_equal(ct[:got].cpu().numpy().view(np.uint32), cols_o)


def test_get_rows_null_cols_is_a_sizing_call():
    """mbrwt_get_rows with cols == NULL answers the size (MBRWT_ERR_CAPACITY +
    cols_needed) whatever cols_cap says, like the other host-form calls."""
    import ctypes as C
    from genome_graph_annotation_amd import BRWTDevice, _lib as L
    d = BRWTDevice.synthetic(10_000, 100, 0.05, 8, 3)
    rows = np.arange(100, dtype=np.uint64)
    off_h, cols_h = d.get_rows(rows)
    offsets = np.zeros(101, dtype=np.uint64)
    need = C.c_uint64(0)
    st = L.lib().mbrwt_get_rows(d._h, rows.ctypes.data_as(C.POINTER(C.c_uint64)), 100,
                                offsets.ctypes.data_as(C.POINTER(C.c_uint64)), None, 1 << 20, C.byref(need))
    assert st == L.MBRWT_ERR_CAPACITY
    assert need.value == len(cols_h) > 0


# ---- the production tree shape: greedy + relax (scripts/kingsford/convert.sh:24) ----

@pytest.mark.parametrize("relax,n_rows", [(10, 2_000_000), (0, 500_000), (12, 1_000_000)])
def test_synthetic_over_greedy_relaxed_shapes(oracle_mod, relax, n_rows):
    """mbrwt_create_synthetic_shaped over the shape of a greedy (+ relaxed)
    tree (binary_grouping_greedy, partitionings.cpp:148-201; relax,
    BRWT_builders.cpp:166-211): leaves labelled by pre-order index, mapped to
    their columns in the CSR writers.  Every kernel variant vs the oracle's
    independent implementation of the same law, and the exported image vs the
    oracle's tree."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    rng = np.random.default_rng(relax + 1)
    dense = rng.random((4000, 300)) < 0.01
    shape = O.OracleTree.from_dense(dense, "greedy", 2, relax).export()
    dev = BRWTDevice.synthetic_shaped(n_rows, shape, 0.003, 7)
    t = O.OracleTree.topdown_shaped(n_rows, shape, 0.003, 7)
    assert dev.num_relations() == t.num_relations() and dev.num_columns() == 300
    rows = rng.integers(0, n_rows, 100_000).astype(np.uint64)
    _check_rows(t, dev, rows)
    off_s, cols_s = O.topdown_get_rows_shaped(n_rows, shape, 0.003, 7, rows)
    off_d, cols_d = dev.get_rows(rows)
    np.testing.assert_array_equal(off_d, off_s)
    np.testing.assert_array_equal(cols_d, cols_s)
    for j in (0, 17, 299):
        np.testing.assert_array_equal(dev.get_column(j), np.asarray(t.get_column(j), dtype=np.uint64))


# ---- KIND_PACKT: any shape's root children packed to the leaves (k_traverse_ptw) ----

@pytest.mark.parametrize("n,m,d,part,arity,relax", [
    (6000, 200, 0.02, "greedy", 2, 10),           # the production shape (relax 10)
    (6000, 200, 0.02, "greedy", 2, 0),            # binary greedy: subtrees of height 7 (8-level walks)
    (4000, 300, 0.02, "greedy", 2, 2**64 - 1),    # unbounded relax
    (4000, 65, 0.05, "basic", 8, 0),              # a root child that is a leaf (pass-through)
    (4000, 1728, 0.002, "basic", 12, 0),          # 12 root children, arity-12 masks (2 bytes)
    (3000, 256, 0.02, "basic", 16, 0),            # 16 root children of 16 leaves
    (3000, 600, 0.01, "basic", 2, 0),             # a child of height 9 (no PACKT) beside one of height 7
])
def test_packt_layout(oracle_mod, n, m, d, part, arity, relax):
    """KIND_PACKT images (mbrwt_internal.hpp) against the oracle and against
    the same tree without them (MBRWT_PACKT=0): rows under every kernel
    (k_traverse_ptw by default, the lane kernel for the rest), columns, get,
    V/L accounting; a run of dense rows makes blocks spill."""
    O = oracle_mod
    rng = np.random.default_rng(n + m)
    dense = rng.random((n, m)) < d
    if arity > 2 or relax:  # (binary subtrees: 0.3-dense rows give records over 64 bytes)
        dense[n // 3:n // 3 + 12] = rng.random((12, m)) < 0.3
    t = O.OracleTree.from_dense(dense, part, arity, relax)
    pt = _dev(t)
    plain = _with_env("MBRWT_PACKT", "0", lambda: _dev(t))
    if m == 600:  # the 512-column child is too tall: mixed images, general kernels
        assert pt.traverse_kernel() != "k_traverse_ptw"
    else:
        assert pt.traverse_kernel() == "k_traverse_ptw"
        assert pt.device_bytes() != plain.device_bytes()
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 20000)]).astype(np.uint64)
    cols = np.random.default_rng(1).integers(0, m, 12)
    _agree(t, [pt, plain], rows, cols, m)


def test_packt_records_longer_than_a_block(oracle_mod):
    """Fully set rows make records longer than 64 bytes: the host builder
    declines KIND_PACKT for those root children; results as the oracle's."""
    O = oracle_mod
    rng = np.random.default_rng(31)
    n, m = 2000, 400
    dense = rng.random((n, m)) < 0.01
    dense[[3, 1000]] = True
    t = O.OracleTree.from_dense(dense, "greedy", 2, 0)  # binary: a full row is one mask per internal node
    d = _dev(t)
    assert d.traverse_kernel() != "k_traverse_ptw"
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 5000)]).astype(np.uint64)
    _agree(t, [d], rows, [0, 5, 399], m)


@pytest.mark.parametrize("relax,n_rows", [(10, 3_000_000), (0, 1_000_000)])
def test_packt_synthetic_shaped(oracle_mod, relax, n_rows):
    """The generator's KIND_PACKT images over a greedy (+ relaxed) shape
    (synth.hip synth_packt) against the oracle's independent implementation
    of the same law, and against the node-by-node images (MBRWT_PACKT=0)."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    rng = np.random.default_rng(relax + 7)
    dense = rng.random((4000, 500)) < 0.01
    shape = O.OracleTree.from_dense(dense, "greedy", 2, relax).export()
    pt = BRWTDevice.synthetic_shaped(n_rows, shape, 0.003, 11)
    plain = _with_env("MBRWT_PACKT", "0", lambda: BRWTDevice.synthetic_shaped(n_rows, shape, 0.003, 11))
    assert pt.traverse_kernel() == "k_traverse_ptw"
    assert pt.device_bytes() != plain.device_bytes()
    t = O.OracleTree.topdown_shaped(n_rows, shape, 0.003, 11)
    rows = rng.integers(0, n_rows, 100_000).astype(np.uint64)
    _agree(t, [pt, plain], rows, [0, 1, 250, 499], 500)


@pytest.mark.parametrize("partitioner,relax", [("basic", 0), ("greedy", 10)])
def test_device_builder_beyond_2_32_rows(oracle_mod, partitioner, relax):
    """The column builders at Row = uint64_t (binary_matrix.hpp:11): 2^32 +
    3,000 rows x 5 sparse columns built on the device (the description goes
    through the row-sharded create) against the oracle's tree of the same
    columns, on the rows either side of 2^31 and 2^32, every set position and
    random rows."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    n, m = 2**32 + 3000, 5
    W = (n + 63) // 64
    rng = np.random.default_rng(77)
    words = np.zeros((m, W), dtype=np.uint64)
    setpos = []
    for j in range(m):
        pos = np.unique(np.concatenate([rng.integers(0, n, 100_000), rng.integers(2**32 - 50, n, 40)]))
        np.bitwise_or.at(words[j], pos // 64, np.left_shift(np.uint64(1), (pos % 64).astype(np.uint64)))
        setpos.append(pos)
    t = O.OracleTree.from_words(words.ravel(), n, m, partitioner, 2, relax)
    built = BRWTDevice.from_columns(words, n, 2, relax_max_arity=relax, partitioner=partitioner)
    assert built.num_rows() == n and built.num_relations() == t.num_relations()
    edges = []
    for e in (2**31, 2**32, n):
        edges += list(range(e - 6, min(e + 6, n)))
    rows = np.concatenate([np.array(edges), np.concatenate(setpos)[::7], rng.integers(0, n, 50_000)])
    rows = rows.astype(np.uint64)
    off_o, cols_o = t.get_rows(rows)
    off_d, cols_d = built.get_rows(rows)
    np.testing.assert_array_equal(off_d, off_o)
    np.testing.assert_array_equal(cols_d, cols_o)
