"""BinRel-WT(sdsl) oracle (oracle/binrel_wt_oracle.cpp) against the reference's
own tests (tests/test_bin_rel_wt_sdsl.cpp:15-176) and the synthetic row spec.
CPU only."""
import numpy as np
import pytest


def _check(O, dense):
    t = O.OracleWT.from_dense(dense)
    n, m = dense.shape
    assert t.num_rows() == n and t.num_columns() == m and t.num_relations() == int(dense.sum())
    for r in range(n):
        assert t.get_row(r) == np.nonzero(dense[r])[0].tolist()
        for c in range(m):
            assert t.get(r, c) == bool(dense[r, c])
    for c in range(m):
        assert t.get_column(c).tolist() == np.nonzero(dense[:, c])[0].tolist()


def test_empty(oracle_mod):
    e = oracle_mod.OracleWT.empty()
    assert e.num_rows() == 0 and e.num_columns() == 0


@pytest.mark.parametrize("kind", ["zero", "one", "mixed"])
def test_reference_grids(oracle_mod, kind):
    hi = 20 if kind == "zero" else 10
    for m in range(1, hi):
        for n in range(1, hi):
            if kind == "zero":
                dense = np.zeros((n, m), dtype=bool)
            elif kind == "one":
                dense = np.ones((n, m), dtype=bool)
            else:  # first and last columns all zero (test_bin_rel_wt_sdsl.cpp:150-153)
                dense = np.zeros((n, m), dtype=bool)
                for j in range(n):
                    for i in range(1, m - 1):
                        dense[j, i] = (i + j) % 2
            _check(oracle_mod, dense)


@pytest.mark.parametrize("n,m,d", [(300, 3173, 0.038), (500, 257, 0.1), (200, 2, 0.5), (100, 1, 0.7)])
def test_random(oracle_mod, n, m, d):
    dense = np.random.default_rng(n + m).random((n, m)) < d
    _check(oracle_mod, dense)


def test_unsorted_and_repeated_ids(oracle_mod):
    """Rows are emitted by generate_rows in any order; interval_symbols still
    returns ascending ids.  A repeated id shows the reference's padding zero
    and repeated row (bin_rel_wt_sdsl.cpp:66-82, :85-96)."""
    O = oracle_mod
    t = O.OracleWT.from_csr(np.array([0, 3, 5], dtype=np.uint64), np.array([5, 1, 3, 2, 2], dtype=np.uint32), 6)
    assert t.get_row(0) == [1, 3, 5]
    assert t.get_row(1) == [2, 0]
    assert t.get_column(2).tolist() == [1, 1]
    assert t.get(1, 2) and not t.get(1, 0)


def _mix64(z):
    M = (1 << 64) - 1
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


def test_synthetic_row_spec(oracle_mod):
    """wt_synth_row follows DESIGN.md "BinRel-WT" (re-derived here in Python)."""
    O = oracle_mod
    M = (1 << 64) - 1
    m, d, seed = 300, 0.05, 42
    T = int(d * 2.0**64)
    assert O.lib().wt_synth_threshold(d) == T
    off, cols = O.wt_synth_rows(1000, 20, m, d, seed)
    for i in range(20):
        K = _mix64(seed ^ (((1000 + i + 1) * 0x9E3779B97F4A7C15) & M))
        want = [c for c in range(m) if _mix64((K + c * 0xD1B54A32D192ED03) & M) < T]
        assert cols[off[i]:off[i + 1]].tolist() == want
    off, cols = O.wt_synth_rows(0, 20000, 3173, 0.038, 42)
    assert abs(off[-1] / 20000 - 3173 * 0.038) < 1.0
