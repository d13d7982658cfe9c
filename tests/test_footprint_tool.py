"""tools/footprint_scale.py's exact RRR byte count (the reference's
compressed index size at scale) against the oracle's
oracle_rrr_bytes (sdsl rrr_vector<63> layout) on materialised trees."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def test_rrr_bytes_matches_oracle(oracle_mod):
    O = oracle_mod
    from footprint_scale import tree_rrr_bytes, weighted_freqs
    rng = np.random.default_rng(3)
    for n, m, d, part in ((1000, 17, 0.3, "basic"), (20_000, 60, 0.02, "greedy"), (63 * 64, 9, 0.5, "basic"),
                          (5, 3, 1.0, "basic")):
        t = O.OracleTree.from_dense(rng.random((n, m)) < d, part, 2)
        plain, rrr = tree_rrr_bytes(t.export())
        assert rrr == t.rrr_bytes()
        assert plain == t.total_column_size() // 8 or abs(plain - t.total_column_size() / 8) < len(t.export()["vec_size"])
    w, nr = O.generate_uniform_rows(30_000, 200, 0.01, 300, 42)
    t = O.OracleTree.from_words(w, nr, 200, "greedy", 2, 10)
    assert tree_rrr_bytes(t.export())[1] == t.rrr_bytes()
    f = weighted_freqs(1_000_000, 10_000)
    assert f[0] == max(f) and f.min() >= 1 and abs(int(f.sum()) - 1_000_000) < 10_000
