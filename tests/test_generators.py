"""The reference's correlated-matrix generators restated in the oracle
(experiments/main.cpp:232-264 uniform_rows / uniform_columns over
data_generation.cpp:66-165: generate, replicate, std::shuffle with the same
mt19937) and the sdsl-RRR size accounting used by tools/footprint.py."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _bits(words, n, m):
    W = (n + 63) // 64
    return np.unpackbits(words.view(np.uint8), bitorder="little").reshape(m, W * 64)[:, :n]


def test_uniform_rows(oracle_mod):
    O = oracle_mod
    words, n = O.generate_uniform_rows(3000, 90, 0.1, 60, 42)
    assert n == 3000
    rows, counts = np.unique(_bits(words, n, 90).T, axis=0, return_counts=True)
    assert len(rows) <= 60 and set(counts.tolist()) <= {50, 100, 150}  # (two drawn rows may coincide)
    # the distinct rows are the generated columns over 60 rows, transposed
    gen = _bits(O.generate_columns(60, 90, 0.1, 42), 60, 90).T
    assert {r.tobytes() for r in rows} == {r.tobytes() for r in gen}
    # not left in generation order
    assert not np.array_equal(_bits(words, n, 90).T[:50], np.repeat(gen[:1], 50, axis=0))


def test_uniform_columns(oracle_mod):
    O = oracle_mod
    words, m = O.generate_uniform_columns(4000, 95, 0.05, 19, 42)
    assert m == 95
    cols = _bits(words, 4000, m)
    uniq, counts = np.unique(cols, axis=0, return_counts=True)
    assert len(uniq) == 19 and set(counts.tolist()) == {5}
    gen = _bits(O.generate_columns(4000, 19, 0.05, 42), 4000, 19)
    assert {c.tobytes() for c in uniq} == {c.tobytes() for c in gen}


def test_rrr_size_model_matches_exact(oracle_mod):
    O = oracle_mod
    import footprint as F
    n, m, d = 400_000, 2652, 0.003
    t = O.OracleTree.topdown(n, m, d, 8, 42)
    exact = t.rrr_bytes()
    model = sum(F.rrr_expected_bytes(sz, p) for sz, p in F.law_nodes(t.export(), n, m, d))
    assert abs(model / exact - 1) < 0.01
    assert exact < t.total_column_size() // 8  # compressed below the plain bits at this density
