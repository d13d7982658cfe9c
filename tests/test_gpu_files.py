"""Device image -> tree description (mbrwt_tree_export) and the reference's
BRWT stream into HBM (mbrwt_load): every image layout decodes back to the
exact index columns it was built from, and a dumped / reloaded matrix answers
every query like the oracle (test_BRWT.cpp:214-238, on the device)."""
import os

import numpy as np
import pytest

from conftest import gpu_available

# the per-node images (the library default, AUTO, builds row records:
# tests/test_gpu_rows.py); a test passing layout= explicitly overrides it
pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU"),
              pytest.mark.usefixtures("nodes_layout")]


def _same_tree(a, b):
    from test_brwt_files import _same_tree as same
    same(a, b)


def _env(name, value, fn):
    """fn() under the build option that replaced the r04 switch `name`."""
    from conftest import with_build
    return with_build(name, value, fn)


@pytest.mark.parametrize("layout", [{}, {"MBRWT_PACK2": "0"}, {"MBRWT_PACK": "0"}, {"MBRWT_FOLD_ROOT": "0"},
                                    {"MBRWT_PACKT": "0"}])
def test_export_every_layout(oracle_mod, layout):
    """PLANE, MASK8..64, PACK (with spilled blocks), PACK2 (with spilled
    blocks), folded and unfolded roots: the exported description is the one
    the image was built from."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    rng = np.random.default_rng(21)
    cases = []
    for n, m, d, part, arity, relax in [(4000, 256, 0.004, "basic", 4, 0), (4000, 64, 0.01, "basic", 8, 0),
                                        (3000, 2048, 0.04, "basic", 8, 0), (2000, 100, 0.05, "greedy", 2, 0),
                                        (2000, 300, 0.02, "basic", 2, 2**64 - 1), (1500, 40, 0.3, "basic", 12, 0),
                                        (1000, 90, 0.02, "basic", 40, 0), (3000, 200, 0.02, "greedy", 2, 10),
                                        (2000, 65, 0.05, "basic", 8, 0), (2000, 256, 0.02, "basic", 16, 0)]:
        dense = rng.random((n, m)) < d
        dense[n // 2:n // 2 + 24] = True  # dense rows: spilled PACK / PACK2 blocks
        cases.append(O.OracleTree.from_dense(dense, part, arity, relax))
    for t in cases:
        exp = t.export()

        def mk():
            return BRWTDevice.from_tree(exp)
        k, v = next(iter(layout.items())) if layout else (None, None)
        dev = _env(k, v, mk) if k else mk()
        _same_tree(exp, dev.export())


def test_export_reference_grids(oracle_mod):
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    for n in range(1, 20, 3):
        for m in range(1, 20, 2):
            i = np.arange(n)[:, None]
            j = np.arange(m)[None, :]
            for dense in (np.zeros((n, m), bool), np.ones((n, m), bool), ((i + 2 * j) % 2).astype(bool)):
                exp = O.OracleTree.from_dense(dense, "basic", 2).export()
                _same_tree(exp, BRWTDevice.from_tree(exp).export())


@pytest.mark.parametrize("n,m,d,arity", [(300_000, 2652, 0.003, 8), (100_000, 3173, 0.038, 8), (50_000, 500, 0.01, 2)])
def test_export_synthetic_images(oracle_mod, n, m, d, arity):
    """The device generator's images (synth.hip) decode to the oracle's
    independent implementation of the same spec."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    dev = BRWTDevice.synthetic(n, m, d, arity, 42)
    _same_tree(O.OracleTree.topdown(n, m, d, arity, 42).export(), dev.export())


@pytest.mark.parametrize("relax", [10, 0])
def test_export_synthetic_packt_images(oracle_mod, relax):
    """KIND_PACKT images of the generator over a greedy (+ relaxed) shape
    decode to the oracle's tree of the same law."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    dense = np.random.default_rng(relax).random((3000, 300)) < 0.01
    shape = O.OracleTree.from_dense(dense, "greedy", 2, relax).export()
    dev = BRWTDevice.synthetic_shaped(400_000, shape, 0.003, 5)
    assert dev.traverse_kernel() == "k_traverse_ptw"
    _same_tree(O.OracleTree.topdown_shaped(400_000, shape, 0.003, 5).export(), dev.export())


def test_dump_and_load_answers_like_the_oracle(oracle_mod):
    """test_BRWT.cpp:214-238 on the device: serialize, load the bytes back into
    HBM, and every row / column / point query is the oracle's."""
    from genome_graph_annotation_amd import BRWTDevice, MBRWTError
    O = oracle_mod
    rng = np.random.default_rng(3)
    n, m = 20_000, 700
    dense = rng.random((n, m)) < 0.01
    t = O.OracleTree.from_dense(dense, "greedy", 2, 8)
    dev = BRWTDevice.from_tree(t.export())
    data = dev.serialize()
    loaded = BRWTDevice.load(data)
    assert loaded.num_rows() == n and loaded.num_columns() == m
    assert loaded.num_relations() == int(dense.sum())
    rows = np.arange(n, dtype=np.uint64)
    off_o, cols_o = t.get_rows(rows)
    off_d, cols_d = loaded.get_rows(rows)
    np.testing.assert_array_equal(off_d, off_o)
    np.testing.assert_array_equal(cols_d, cols_o)
    for j in range(0, m, 37):
        np.testing.assert_array_equal(loaded.get_column(j), np.asarray(t.get_column(j), dtype=np.uint64))
    with pytest.raises(MBRWTError):
        BRWTDevice.load(data[: len(data) // 2])
    # a synthetic Kingsford-shaped matrix survives the dump too
    syn = BRWTDevice.synthetic(200_000, 2652, 0.003, 8, 9)
    back = BRWTDevice.load(syn.serialize())
    q = rng.integers(0, 200_000, 50_000).astype(np.uint64)
    a, b = syn.get_rows(q), back.get_rows(q)
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])


# ---- row-record contexts (layout rows; the library default AUTO picks them) --

def _rows_cases(O, rng):
    out = []
    for n, m, d, part, arity, relax in [(4000, 256, 0.004, "basic", 4, 0), (4000, 64, 0.01, "basic", 8, 0),
                                        (3000, 2048, 0.04, "basic", 8, 0), (2000, 100, 0.05, "greedy", 2, 0),
                                        (3000, 200, 0.02, "greedy", 2, 10), (1500, 40, 0.3, "basic", 12, 0),
                                        (2000, 256, 0.02, "basic", 16, 0), (1000, 7, 1.0, "basic", 2, 0),
                                        (1000, 9, 0.0, "basic", 3, 0)]:
        dense = rng.random((n, m)) < d
        dense[n // 2:n // 2 + 24] = True  # dense rows: spilled entries, records longer than a block
        out.append((dense, O.OracleTree.from_dense(dense, part, arity, relax)))
    return out


def test_export_rows_layout(oracle_mod):
    """mbrwt_tree_export of a row-record context (no node image): the index
    columns rebuilt from the records are the ones the context was built from,
    for every block shape the builder picks (spills and long rows included)."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    for dense, t in _rows_cases(O, np.random.default_rng(22)):
        exp = t.export()
        dev = BRWTDevice.from_tree(exp, layout="rows")
        assert dev.layout() == "rows"
        _same_tree(exp, dev.export())


def test_export_rows_ranged_and_synthetic(oracle_mod):
    """Export of a ranged row-record build (several ranges of rows, the
    synthetic law across them) equals the oracle's tree of the same spec."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    dev = _env("MBRWT_ROWS_RANGE", "360360", lambda: BRWTDevice.synthetic(1_100_000, 700, 0.004, 8, 9, layout="rows"))
    _same_tree(O.OracleTree.topdown(1_100_000, 700, 0.004, 8, 9).export(), dev.export())
    syn = BRWTDevice.synthetic(300_000, 2652, 0.003, 8, 42, layout="rows")
    _same_tree(O.OracleTree.topdown(300_000, 2652, 0.003, 8, 42).export(), syn.export())


def test_rows_serialize_round_trip(oracle_mod):
    """BinaryMatrix::serialize of a row-record context (BRWT.cpp:113-128)
    loads back through mbrwt_load (BRWT.cpp:87-111) -- into the default
    layout -- and answers like the oracle (test_BRWT.cpp:214-238)."""
    from genome_graph_annotation_amd import BRWTDevice
    O = oracle_mod
    rng = np.random.default_rng(4)
    for dense, t in _rows_cases(O, rng)[:5]:
        n, m = dense.shape
        dev = BRWTDevice.from_tree(t.export(), layout="rows")
        data = dev.serialize()
        assert data == BRWTDevice.from_tree(t.export(), layout="nodes").serialize()
        for layout in ("rows", None):
            back = BRWTDevice.load(data, layout=layout)
            rows = np.arange(n, dtype=np.uint64)
            off_o, cols_o = t.get_rows(rows)
            off_d, cols_d = back.get_rows(rows)
            np.testing.assert_array_equal(off_d, off_o)
            np.testing.assert_array_equal(cols_d, cols_o)
            for j in sorted({0, m - 1, int(rng.integers(0, m))}):
                np.testing.assert_array_equal(back.get_column(j), np.asarray(t.get_column(j), dtype=np.uint64))
