"""Pins the CPU oracle to the reference's own known-answer tests.

The reference's tests (GoogleTest, not runnable here: sdsl-lite is absent)
are restated case by case:
  tests/test_bit_vector.cpp:19-94      rank/select identities, clamping, 16-bit KAT
  tests/test_BRWT.cpp:15-212           shapes, arity, all grids 1..19 x 1..19
  tests/test_BRWT_optimizer.cpp:15-163 the same after relax
plus the generator semantics of experiments/data_generation.cpp.
"""
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def reference_based_test(O, bits):  # test_bit_vector.cpp:19-47
    v = O.BitVec(bits)
    max_rank = int(np.sum(bits))
    for i in (1, 2, 10, 100, 1000):
        assert v.rank1(v.size + i - 2) == max_rank  # clamping
        with pytest.raises(IndexError):
            v.select1(max_rank + i)
    with pytest.raises(IndexError):
        v.select1(0)
    for i in range(1, max_rank + 1):
        assert v.rank1(v.select1(i)) == i
    assert v[0] == v.rank1(0) == bits[0]
    for i in range(1, v.size):
        assert v[i] == v.rank1(i) - v.rank1(i - 1) == bits[i]


def test_bit_vector_queries(oracle_mod):  # test_bit_vector.cpp:50-94
    O = oracle_mod
    z = O.BitVec([0] * 10)
    for i in range(10):
        assert z[i] == 0 and z.rank1(i) == 0
        with pytest.raises(IndexError):
            z.select1(i)
    assert z.rank1(1000) == 0
    o = O.BitVec([1] * 10)
    for i in range(10):
        assert o[i] == 1 and o.select1(i + 1) == i and o.rank1(i) == i + 1
        assert o.rank1(o.select1(i + 1)) == i + 1 and o.select1(o.rank1(i)) == i
    assert o.rank1(1000) == 10
    kat = json.load(open(os.path.join(GOLDEN, "kat_bitvector.json")))
    reference_based_test(O, kat["bits"])
    v = O.BitVec(kat["bits"])
    assert [v.rank1(i) for i in range(16)] == kat["rank1"]
    assert [v.select1(i + 1) for i in range(kat["total"])] == kat["select1_1based"]
    rng = np.random.default_rng(0)
    for n in (1, 63, 64, 65, 511, 512, 513, 5000):
        reference_based_test(O, (rng.random(n) < 0.3).astype(int).tolist())


def test_brwt_shapes(oracle_mod):  # test_BRWT.cpp:15-90
    O = oracle_mod
    e = O.OracleTree.from_dense(np.zeros((0, 0), dtype=bool))
    assert e.num_columns() == 0 and e.num_rows() == 0 and e.num_nodes() == 1 and e.avg_arity() == 0
    one = O.OracleTree.from_dense(np.ones((10, 1), dtype=bool))
    assert one.num_columns() == 1 and one.num_rows() == 10 and one.num_nodes() == 1 and one.avg_arity() == 0
    zero = O.OracleTree.from_dense(np.zeros((10, 1), dtype=bool))
    assert zero.num_nodes() == 1 and zero.avg_arity() == 0
    for cols in ([1, 0], [0, 1]):
        t = O.OracleTree.from_dense(np.array([cols] * 10, dtype=bool))
        assert t.num_nodes() == 3 and t.avg_arity() == 2
        r = O.OracleTree.from_dense(np.array([cols] * 10, dtype=bool), relax=2**64 - 1)
        assert r.num_nodes() == 3 and r.avg_arity() == 2


def _grid(kind, n, m):
    if kind == "zero":
        return np.zeros((n, m), dtype=bool)
    if kind == "one":
        return np.ones((n, m), dtype=bool)
    return ((np.arange(n)[:, None] + 2 * np.arange(m)[None, :]) % 2).astype(bool)


def _test_brwt(t, dense):  # test_BRWT.cpp:92-150
    n, m = dense.shape
    assert t.num_columns() == m and t.num_rows() == n
    for j in range(m):
        col = t.get_column(j)
        assert len(col) == len(set(col)) == int(dense[:, j].sum())
        assert all(dense[i, j] for i in col)
    for i in range(n):
        row = t.get_row(i)
        assert len(row) == len(set(row))
        assert set(row) == set(np.nonzero(dense[i])[0].tolist())
    for i in range(n):
        for j in range(m):
            assert t.get(i, j) == dense[i, j]


@pytest.mark.parametrize("relax", [0, 2**64 - 1])
@pytest.mark.parametrize("kind", ["zero", "one", "mixed"])
def test_brwt_grids(oracle_mod, kind, relax):  # test_BRWT.cpp:152-212, test_BRWT_optimizer.cpp:102-163
    O = oracle_mod
    for n in range(1, 20):
        for m in range(1, 20):
            dense = _grid(kind, n, m)
            t = O.OracleTree.from_dense(dense, "basic", 2, relax)
            assert t.num_relations() == int(dense.sum())
            if kind == "mixed" and not relax:
                assert t.avg_arity() <= 2
            _test_brwt(t, dense)


def test_basic_partitioner_order_and_shape(oracle_mod):
    """Basic arity-k partitioner: rows come back ascending (BRWT_builders.cpp:24-30, :84-91);
    Kingsford shape: levels 2652 -> 332 -> 42 -> 6 -> 1."""
    O = oracle_mod
    rng = np.random.default_rng(1)
    dense = rng.random((300, 77)) < 0.2
    for arity in (2, 3, 5, 8):
        t = O.OracleTree.from_dense(dense, "basic", arity)
        for i in range(300):
            assert t.get_row(i) == np.nonzero(dense[i])[0].tolist()
    t = O.OracleTree.topdown(1000, 2652, 0.003, 8, 1)
    assert t.num_nodes() == 2652 + 332 + 42 + 6 + 1 and t.depth() == 5


def test_generate_random_ints_semantics(oracle_mod):
    """experiments/data_generation.cpp:7-18: std::uniform_int_distribution<int>
    on a DataGenerator seeded 42 -- deterministic, within [begin, end)."""
    O = oracle_mod
    a = O.generate_random_ints(1000, 0, 1_000_000, 42)
    b = O.generate_random_ints(1000, 0, 1_000_000, 42)
    assert np.array_equal(a, b) and a.min() >= 0 and a.max() < 1_000_000
    assert not np.array_equal(a, O.generate_random_ints(1000, 0, 1_000_000, 43))


def test_norepl_generator_density(oracle_mod):
    """data_generation.cpp:20-29: one Bernoulli(d) draw per cell, column-major."""
    O = oracle_mod
    n, m, d = 20000, 50, 0.01
    w = O.generate_columns(n, m, d, 42)
    ones = int(np.unpackbits(w.view(np.uint8)).sum())
    assert abs(ones / (n * m) - d) < 4 * np.sqrt(d / (n * m))
    t = O.OracleTree.norepl(n, m, d, 42, "basic", 2)
    assert t.num_relations() == ones


def test_topdown_law_matches_iid_columns(oracle_mod):
    """The top-down generator draws the law of a BRWT over i.i.d. Bernoulli(d)
    columns: compare the node-level densities and label counts with a BRWT
    built bottom-up from actual i.i.d. columns (reference generator)."""
    O = oracle_mod
    n, m, d = 200_000, 64, 0.01
    td = O.OracleTree.topdown(n, m, d, 8, 5)
    bu = O.OracleTree.norepl(n, m, d, 42, "basic", 8)
    for a, b in ((td.num_relations(), bu.num_relations()), (td.total_num_set_bits(), bu.total_num_set_bits()),
                 (td.total_column_size(), bu.total_column_size())):
        assert abs(a - b) / b < 0.02, (a, b)
    rows = np.arange(0, n, 7, dtype=np.uint64)
    _, c1, v1 = td.get_rows(rows, with_visits=True)
    _, c2, v2 = bu.get_rows(rows, with_visits=True)
    assert abs(len(c1) - len(c2)) / len(c2) < 0.03
    assert abs(v1.mean() - v2.mean()) / v2.mean() < 0.02
    # BRWT invariant: every set parent bit has at least one set child (checked
    # through get_row: a row with a set root bit has at least one label)
    for r in range(0, 2000):
        assert (len(td.get_row(r)) > 0) == bool(td.get(r, 0) or any(td.get(r, j) for j in range(m)))


def test_kingsford_work_per_row(oracle_mod):
    """V ~ 159.5 probes and L ~ 7.96 labels per row at the Kingsford shape."""
    O = oracle_mod
    t = O.OracleTree.topdown(300_000, 2652, 0.003, 8, 42)
    _, cols, v = t.get_rows(np.arange(0, 300_000, 3, dtype=np.uint64), with_visits=True)
    assert abs(v.mean() - 159.5) < 1.5
    assert abs(len(cols) / len(v) - 7.96) < 0.15
