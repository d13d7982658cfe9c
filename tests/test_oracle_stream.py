"""The streamed top-down oracle (oracle.topdown_get_rows, used by the
full-size parity checks) against the materialised oracle tree of the same
spec: identical CSR (BRWT::get_row, BRWT.cpp:26-53) for shapes with
pass-through leaves, one column, arities 2..12, repeated and unsorted rows,
and the out-of-range error.  CPU only."""
import numpy as np
import pytest


@pytest.mark.parametrize("n,m,d,arity", [
    (1000, 1, 0.3, 8), (5000, 9, 0.1, 8), (20000, 65, 0.02, 8), (50000, 500, 0.01, 2),
    (100000, 2652, 0.003, 8), (30000, 3173, 0.038, 8), (10000, 17, 0.2, 4), (3000, 130, 0.05, 3),
    (4000, 300, 0.05, 12), (2000, 40, 0.0, 8), (2000, 40, 1.0, 8),
])
def test_stream_matches_materialised_tree(oracle_mod, n, m, d, arity):
    O = oracle_mod
    rows = np.random.default_rng(n + m).integers(0, n, 20000).astype(np.uint64)
    rows[:50] = rows[50]  # repeats
    rows[-1] = n - 1
    t = O.OracleTree.topdown(n, m, d, arity, 42)
    o1, c1 = t.get_rows(rows)
    o2, c2 = O.topdown_get_rows(n, m, d, arity, 42, rows)
    assert np.array_equal(o1, o2)
    assert np.array_equal(c1, c2)


def test_stream_edges(oracle_mod):
    O = oracle_mod
    off, cols = O.topdown_get_rows(100, 10, 0.1, 8, 1, np.zeros(0, dtype=np.uint64))
    assert off.tolist() == [0] and len(cols) == 0
    with pytest.raises(IndexError):
        O.topdown_get_rows(100, 10, 0.1, 8, 1, np.array([100], dtype=np.uint64))


def test_wt_rows_at_matches_range(oracle_mod):
    O = oracle_mod
    o1, c1 = O.wt_synth_rows(0, 3000, 500, 0.05, 7)
    rows = np.random.default_rng(3).integers(0, 3000, 5000).astype(np.uint64)
    o2, c2 = O.wt_synth_rows_at(rows, 500, 0.05, 7)
    for i, r in enumerate(rows[:500]):
        assert np.array_equal(c2[o2[i]:o2[i + 1]], c1[o1[r]:o1[r + 1]])
    assert o2[-1] == sum(o1[r + 1] - o1[r] for r in rows)


@pytest.mark.parametrize("n,m,d,arity", [(50000, 2652, 0.003, 8), (20000, 3173, 0.038, 8), (3000, 9, 0.5, 2),
                                         (20000, 50, 0.9, 2), (3000, 7, 0.0, 2), (3000, 7, 1.0, 2), (4033, 5, 0.97, 2)])
def test_rrr_layout_answers_like_plain(oracle_mod, n, m, d, arity):
    """The CPU baseline's sdsl-RRR-like index vectors (oracle_to_rrr) give the
    plain vectors' get_row / get / V accounting exactly."""
    O = oracle_mod
    t = O.OracleTree.topdown(n, m, d, arity, 42)
    rows = np.random.default_rng(n).integers(0, n, 5000).astype(np.uint64)
    o1, c1, v1 = t.get_rows(rows, with_visits=True)
    pts = [(int(r), int(c)) for r, c in zip(rows[:300], np.random.default_rng(1).integers(0, m, 300))]
    g1 = [t.get(r, c) for r, c in pts]
    t.to_rrr()
    o2, c2, v2 = t.get_rows(rows, with_visits=True)
    assert np.array_equal(o1, o2) and np.array_equal(c1, c2) and np.array_equal(v1, v2)
    assert g1 == [t.get(r, c) for r, c in pts]


@pytest.mark.parametrize("part,arity,relax", [("greedy", 2, 10), ("greedy", 2, 0), ("basic", 3, 0)])
def test_shaped_stream_matches_shaped_tree(oracle_mod, part, arity, relax):
    """The top-down law over an arbitrary shape (a greedy + relaxed tree's, the
    reference's production build path): streamed query == materialised tree."""
    O = oracle_mod
    rng = np.random.default_rng(arity + relax)
    dense = rng.random((3000, 70)) < 0.02
    shape = O.OracleTree.from_dense(dense, part, arity, relax).export()
    N = 1_000_000
    t = O.OracleTree.topdown_shaped(N, shape, 0.01, 42)
    rows = rng.integers(0, N, 20000).astype(np.uint64)
    o1, c1 = t.get_rows(rows)
    o2, c2 = O.topdown_get_rows_shaped(N, shape, 0.01, 42, rows)
    assert np.array_equal(o1, o2) and np.array_equal(c1, c2)
    assert t.num_columns() == 70


def test_shaped_law_on_the_basic_shape_is_the_basic_law(oracle_mod):
    O = oracle_mod
    t = O.OracleTree.topdown(100000, 2652, 0.003, 8, 42)
    t2 = O.OracleTree.topdown_shaped(100000, t.export(), 0.003, 42)
    rows = np.random.default_rng(5).integers(0, 100000, 20000).astype(np.uint64)
    a, b = t.get_rows(rows), t2.get_rows(rows)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
