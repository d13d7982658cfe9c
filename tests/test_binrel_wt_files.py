"""BinRelWT_sdsl's stream (load / serialize, bin_rel_wt_sdsl.cpp:113-132)
through libmbrwt's host-side reader and writer (include/mbrwt_wt.h; no GPU).

The stream is {libmaus2 number num_columns, sdsl wt_int<rrr_vector<63>> of
the rows' ids concatenated, bit_vector_rrr delimiters}.  sdsl-lite is an empty
submodule here and the reference holds no written file, so the byte layout is
PARITY UNPINNED: these tests pin the round trip, the framing
rules the reference's own code states (a 1, then per row a 0 per id and a 1:
the ctor, bin_rel_wt_sdsl.cpp:16-34) and the rejection of malformed streams
(load returns false: :113-122).
"""
import numpy as np
import pytest

from genome_graph_annotation_amd import MBRWTError, _lib as L
from genome_graph_annotation_amd.binrel_wt import parse_stream, serialize_csr


def _random_csr(rng, n, m, d):
    dense = rng.random((n, m)) < d
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(dense.sum(1), out=off[1:])
    return off, np.nonzero(dense)[1].astype(np.uint32)


@pytest.mark.parametrize("n,m,d", [(0, 5, 0.0), (1, 1, 1.0), (7, 3, 0.5), (200, 1000, 0.01), (500, 64, 0.3),
                                   (1000, 70000, 0.0005), (64, 2, 0.0)])
def test_round_trip(n, m, d):
    rng = np.random.default_rng(n + m)
    off, cols = _random_csr(rng, n, m, d)
    data = serialize_csr(off, cols, m)
    off2, cols2, m2, used = parse_stream(data)
    assert used == len(data) and m2 == m
    np.testing.assert_array_equal(off2, off)
    np.testing.assert_array_equal(cols2, cols)
    # libmaus2 number: 8 bytes, most significant first
    assert int.from_bytes(data[:8], "big") == m
    # wt_int header: u64 size (the relations), u64 sigma (distinct ids)
    assert int.from_bytes(data[8:16], "little") == len(cols)
    assert int.from_bytes(data[16:24], "little") == len(np.unique(cols))


def test_unsorted_rows_keep_their_order():
    """The writer keeps the order generate_rows emits (flat[index++] =
    col_index, bin_rel_wt_sdsl.cpp:27-28); the reader returns it verbatim."""
    off = np.array([0, 3, 3, 5], dtype=np.uint64)
    cols = np.array([9, 2, 5, 1, 0], dtype=np.uint32)
    off2, cols2, m, _ = parse_stream(serialize_csr(off, cols, 10))
    np.testing.assert_array_equal(off2, off)
    np.testing.assert_array_equal(cols2, cols)


def test_bad_streams_are_rejected():
    rng = np.random.default_rng(3)
    off, cols = _random_csr(rng, 60, 40, 0.1)
    data = serialize_csr(off, cols, 40)
    for cut in range(0, len(data), max(1, len(data) // 97)):
        with pytest.raises(MBRWTError) as ei:
            parse_stream(data[:cut])
        assert ei.value.status == L.MBRWT_ERR_INVALID
    # ids >= num_columns
    bad = bytearray(data)
    bad[:8] = (3).to_bytes(8, "big")
    with pytest.raises(MBRWTError):
        parse_stream(bytes(bad))
    # huge size fields anywhere in the stream: an error, never a crash
    for off_b in range(0, len(data) - 8, 3):
        b = bytearray(data)
        b[off_b:off_b + 8] = (2**64 - 1).to_bytes(8, "little")
        try:
            parse_stream(bytes(b))
        except MBRWTError as e:
            assert e.status == L.MBRWT_ERR_INVALID


def test_writer_rejects_out_of_range_ids():
    with pytest.raises(MBRWTError) as ei:
        serialize_csr(np.array([0, 1], dtype=np.uint64), np.array([5], dtype=np.uint32), 5)
    assert ei.value.status == L.MBRWT_ERR_RANGE
