"""Generates the committed golden fixtures under tests/golden/.

The reference cannot be built here (sdsl-lite / libmaus2 are absent), so the
fixtures come from the oracle (oracle/brwt_oracle.cpp, a restatement of
BRWT.cpp:26-53 on the reference's own builder and generator), and every
fixture is also checked here against its dense ground truth (the matrix the
generator drew), which pins the oracle independently of its own code:
row i's labels must be exactly the set columns of row i.

Run from the repo root:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402


def dense_from_words(words, n, m):
    W = (n + 63) // 64
    bits = np.unpackbits(words.view(np.uint8).reshape(m, W * 8), axis=1, bitorder="little")[:, :n]
    return bits.T.astype(bool)


def check_against_dense(dense, rows, off, cols, ordered_ascending):
    for k, r in enumerate(rows):
        got = cols[off[k]:off[k + 1]].tolist()
        want = np.nonzero(dense[r])[0].tolist()
        assert sorted(got) == want, (k, r)
        if ordered_ascending:
            assert got == want


def norepl_fixture(name, n, m, d, arity, nq, partitioner="basic"):
    words = O.generate_columns(n, m, d, 42)
    dense = dense_from_words(words, n, m)
    t = O.OracleTree.norepl(n, m, d, 42, partitioner, arity)
    rows = O.generate_random_ints(nq, 0, n, 42)  # experiments/main.cpp:78-93
    off, cols, vis = t.get_rows(rows, with_visits=True)
    check_against_dense(dense, rows, off, cols, partitioner == "basic")
    np.savez_compressed(os.path.join(HERE, name), n=n, m=m, d=d, arity=arity, seed=42, rows=rows, offsets=off,
                        cols=cols, visits=vis, num_relations=t.num_relations(), num_nodes=t.num_nodes(),
                        partitioner=partitioner)
    print(name, "rows", nq, "labels", len(cols), "relations", t.num_relations())


def dense_fixture(name, n, m, d, partitioner, arity, relax, seed):
    dense = np.random.default_rng(seed).random((n, m)) < d
    t = O.OracleTree.from_dense(dense, partitioner, arity, relax)
    rows = np.arange(n, dtype=np.uint64)
    off, cols = t.get_rows(rows)
    check_against_dense(dense, rows, off, cols, partitioner == "basic")
    np.savez_compressed(os.path.join(HERE, name), dense=np.packbits(dense, axis=1), n=n, m=m, rows=rows,
                        offsets=off, cols=cols, partitioner=partitioner, arity=arity, relax=relax)
    print(name, "labels", len(cols))


def synth_fixture(name, n, m, d, arity, nq):
    t = O.OracleTree.topdown(n, m, d, arity, 42)
    rows = np.random.default_rng(7).integers(0, n, nq, dtype=np.uint64)
    off, cols, vis = t.get_rows(rows, with_visits=True)
    hashes = [O.synth_hash(42, k, p) for k in (0, 1, 0xFFFFFFFF) for p in (0, 1, 12345, 2**32 - 1)]
    np.savez_compressed(os.path.join(HERE, name), n=n, m=m, d=d, arity=arity, seed=42, rows=rows, offsets=off,
                        cols=cols, visits=vis, num_relations=t.num_relations(),
                        hashes=np.array(hashes, dtype=np.uint64))
    print(name, "labels", len(cols), "relations", t.num_relations())


def bitvector_kat():
    # tests/test_bit_vector.cpp:87-92: the 16-bit known-answer vector; the
    # expected rank/select tables are computed here from the definitions
    # (bit_vector.hpp:16-20: inclusive rank, 1-based select, clamping)
    v = [0, 1, 0, 1, 1, 1, 1, 0, 0, 1, 0, 0, 0, 0, 1, 1]
    rank = [int(sum(v[: i + 1])) for i in range(len(v))]
    select = [i for i, b in enumerate(v) if b]
    with open(os.path.join(HERE, "kat_bitvector.json"), "w") as f:
        json.dump({"bits": v, "rank1": rank, "select1_1based": select, "total": sum(v)}, f, indent=1)
    print("kat_bitvector.json")


if __name__ == "__main__":
    bitvector_kat()
    # BASELINE configs[0] shape class (500 columns, arity 2) at one of its densities
    norepl_fixture("c1_norepl_small.npz", 20000, 500, 0.01 * 7 / 12, 2, 1000)
    # BASELINE configs[1] shape class (2,652 columns, d=0.3%, arity 8)
    norepl_fixture("c2_kingsford_small.npz", 20000, 2652, 0.003, 8, 2000)
    # greedy pairing: output is NOT ascending (partitionings.cpp:159-187)
    dense_fixture("greedy_relax_small.npz", 3000, 40, 0.1, "greedy", 2, 4, 11)
    dense_fixture("basic_relax_unbounded.npz", 2000, 100, 0.05, "basic", 2, 2**64 - 1, 12)
    # the top-down synthetic generator (DESIGN.md "Synthetic matrices")
    synth_fixture("synth_kingsford_small.npz", 200000, 2652, 0.003, 8, 5000)
