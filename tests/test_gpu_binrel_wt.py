"""GPU parity of the BinRel-WT engine (include/mbrwt_wt.h) against the
BinRel-WT(sdsl) oracle: get_row / get / get_column, bit-exact (integer work,
no tolerance).  Cases: the reference's grids (test_bin_rel_wt_sdsl.cpp:86-176),
random matrices over 1..3,173 columns (several chunks, 1..12-bit symbols),
unsorted input rows, error and capacity paths, and the device-generated
synthetic matrix against the oracle's independent generator."""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def _compare(O, t, d, rows=None, cols=None):
    n = t.num_rows()
    assert d.num_rows() == n and d.num_columns() == t.num_columns() and d.num_relations() == t.num_relations()
    rows = np.arange(n, dtype=np.uint64) if rows is None else rows
    off_o, cols_o = t.get_rows(rows)
    off_d, cols_d = d.get_rows(rows)
    np.testing.assert_array_equal(off_d, off_o)
    np.testing.assert_array_equal(cols_d, cols_o)
    m = t.num_columns()
    for c in (range(m) if cols is None else cols):
        np.testing.assert_array_equal(d.get_column(int(c)), t.get_column(int(c)), err_msg=f"column {c}")
    return off_o, cols_o


@pytest.mark.parametrize("kind", ["zero", "one", "mixed"])
def test_reference_grids(oracle_mod, kind):
    from genome_graph_annotation_amd import BinRelWTDevice
    O = oracle_mod
    hi = 20 if kind == "zero" else 10
    for m in range(1, hi, 2):
        for n in range(1, hi, 3):
            if kind == "zero":
                dense = np.zeros((n, m), dtype=bool)
            elif kind == "one":
                dense = np.ones((n, m), dtype=bool)
            else:
                dense = np.zeros((n, m), dtype=bool)
                for j in range(n):
                    for i in range(1, m - 1):
                        dense[j, i] = (i + j) % 2
            t = O.OracleWT.from_dense(dense)
            d = BinRelWTDevice.from_dense(dense)
            _compare(O, t, d)
            ii, jj = np.meshgrid(np.arange(n), np.arange(m), indexing="ij")
            np.testing.assert_array_equal(d.get_batch(ii.ravel(), jj.ravel()), dense.ravel())


@pytest.mark.parametrize("n,m,dens", [
    (3000, 3173, 0.038),   # RefSeq-shaped rows (12-bit symbols)
    (5000, 2652, 0.003),   # Kingsford-shaped rows
    (20000, 1, 0.5),       # 1-bit symbols
    (4000, 2, 0.9),
    (3000, 256, 0.2),      # 8-bit boundary
    (3000, 257, 0.2),      # 9-bit symbols
    (2000, 40, 1.0),       # dense rows
    (1_100_000, 3, 0.4),   # several row chunks (2^k rows per chunk)
])
def test_random_matrices(oracle_mod, n, m, dens):
    from genome_graph_annotation_amd import BinRelWTDevice
    O = oracle_mod
    rng = np.random.default_rng(n + m)
    dense = rng.random((n, m)) < dens
    t = O.OracleWT.from_dense(dense)
    d = BinRelWTDevice.from_dense(dense)
    q = np.concatenate([np.arange(min(n, 3000)), rng.integers(0, n, 20000)]).astype(np.uint64)
    cols = range(m) if m <= 64 else rng.integers(0, m, 24)
    _compare(O, t, d, q, cols)
    qi = rng.integers(0, n, 20000).astype(np.uint64)
    qj = rng.integers(0, m, 20000).astype(np.uint64)
    np.testing.assert_array_equal(d.get_batch(qi, qj), dense[qi.astype(np.int64), qj.astype(np.int64)])


def test_unsorted_rows_errors_and_capacity(oracle_mod):
    import torch
    from genome_graph_annotation_amd import BinRelWTDevice, MBRWTError, _lib as L
    O = oracle_mod
    off = np.array([0, 3, 3, 5], dtype=np.uint64)
    cols = np.array([5, 1, 3, 4, 0], dtype=np.uint32)  # rows emitted unsorted
    t = O.OracleWT.from_csr(off, cols, 6)
    d = BinRelWTDevice.from_csr(off, cols, 6)
    _compare(O, t, d)
    assert d.get_row(0) == [1, 3, 5] and d.get_row(1) == [] and d.get_row(2) == [0, 4]
    with pytest.raises(MBRWTError) as ei:
        d.get_rows([3])
    assert ei.value.status == L.MBRWT_ERR_RANGE
    with pytest.raises(MBRWTError) as ei:
        d.get_batch([0], [6])
    assert ei.value.status == L.MBRWT_ERR_RANGE
    with pytest.raises(MBRWTError) as ei:
        d.get_column(6)
    assert ei.value.status == L.MBRWT_ERR_RANGE
    # rows are sets: a repeated id or an id >= num_columns is rejected
    with pytest.raises(MBRWTError):
        BinRelWTDevice.from_csr(np.array([0, 2], dtype=np.uint64), np.array([2, 2], dtype=np.uint32), 6)
    with pytest.raises(MBRWTError):
        BinRelWTDevice.from_csr(np.array([0, 1], dtype=np.uint64), np.array([6], dtype=np.uint32), 6)
    # device API + capacity protocol
    rt = torch.tensor([2, 0, 1], dtype=torch.int64, device="cuda")
    ot = torch.empty(4, dtype=torch.int64, device="cuda")
    small = torch.empty(2, dtype=torch.int32, device="cuda")
    with pytest.raises(MBRWTError) as ei:
        d.get_rows_device(rt, ot, small)
    assert ei.value.status == L.MBRWT_ERR_CAPACITY and ei.value.needed == 5
    big = torch.empty(8, dtype=torch.int32, device="cuda")
    assert d.get_rows_device(rt, ot, big, torch.cuda.current_stream().cuda_stream) == 5
    torch.cuda.synchronize()
    assert ot.cpu().tolist() == [0, 2, 5, 5]
    assert big[:5].cpu().tolist() == [0, 4, 1, 3, 5]
    e = BinRelWTDevice.from_csr(np.zeros(1, dtype=np.uint64), np.zeros(0, dtype=np.uint32), 0)
    assert e.num_rows() == 0 and e.num_columns() == 0


@pytest.mark.parametrize("n,m,dens", [(300_000, 3173, 0.038), (2_000_000, 2652, 0.003)])
def test_synthetic_matches_oracle(oracle_mod, n, m, dens):
    """The device generator and the oracle's generator draw the same rows;
    the device structure answers like the oracle's BinRel-WT over them."""
    from genome_graph_annotation_amd import BinRelWTDevice
    O = oracle_mod
    d = BinRelWTDevice.synthetic(n, m, dens, 42)
    off, cols = O.wt_synth_rows(0, n, m, dens, 42)
    assert d.num_relations() == int(off[-1])
    rng = np.random.default_rng(7)
    q = rng.integers(0, n, 100_000).astype(np.uint64)
    off_d, cols_d = d.get_rows(q)
    lens = (off[q.astype(np.int64) + 1] - off[q.astype(np.int64)]).astype(np.uint64)
    np.testing.assert_array_equal(np.diff(off_d), lens)
    want = np.concatenate([cols[off[r]:off[r + 1]] for r in q[:5000].astype(np.int64)])
    np.testing.assert_array_equal(cols_d[: len(want)], want)
    if n <= 300_000:  # the oracle's own wavelet tree over the same rows
        t = O.OracleWT.from_csr(off, cols, m)
        _compare(O, t, d, q[:20000], rng.integers(0, m, 8))


@pytest.mark.parametrize("ratio,num_top", [(0.0, 2**64 - 1), (0.5, 3), (1.0, 1)])
def test_classify_batches_over_binrel_wt(oracle_mod, ratio, num_top):
    """mbrwt_wt_get_labels_batch / mbrwt_wt_get_top_labels_batch (the classify
    driver over BinRel-WT rows) against annotate_static.cpp:71-94 and
    annotate.cpp:57-83 on the dense matrix the rows came from (equal counts:
    ascending label), plus the device-buffer form."""
    import math
    import torch
    from genome_graph_annotation_amd import BinRelWTDevice
    rng = np.random.default_rng(int(ratio * 10) + 5)
    n, m = 4000, 300
    dense = rng.random((n, m)) < 0.05
    d = BinRelWTDevice.from_dense(dense)
    lens = rng.integers(0, 30, 500)
    read_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    rows = rng.integers(0, n, int(read_off[-1])).astype(np.uint64)
    lo, labs = d.get_labels_batch(rows, read_off, ratio)
    tlo, tl, tc = d.get_top_labels_batch(rows, read_off, num_top)
    for r in range(len(lens)):
        a, b = int(read_off[r]), int(read_off[r + 1])
        cnt = dense[rows[a:b].astype(np.int64)].sum(axis=0)
        thr = 1 if ratio == 0 else math.ceil((b - a) * ratio)
        np.testing.assert_array_equal(labs[lo[r]:lo[r + 1]], np.nonzero((cnt > 0) & (cnt >= thr))[0])
        nz = np.nonzero(cnt)[0]
        want = nz[np.lexsort((nz, -cnt[nz].astype(np.int64)))][:min(num_top, m)]
        np.testing.assert_array_equal(tl[tlo[r]:tlo[r + 1]], want)
        np.testing.assert_array_equal(tc[tlo[r]:tlo[r + 1]], cnt[want])
    rt = torch.from_numpy(rows.view(np.int64)).cuda()
    ot = torch.from_numpy(read_off.view(np.int64)).cuda()
    lot = torch.empty(len(read_off), dtype=torch.int64, device="cuda")
    lt = torch.empty(max(1, len(labs)), dtype=torch.int32, device="cuda")
    got = d.get_labels_batch_device(rt, ot, ratio, lot, lt, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert got == len(labs)
    np.testing.assert_array_equal(lot.cpu().numpy().view(np.uint64), lo)
    np.testing.assert_array_equal(lt[:got].cpu().numpy().view(np.uint32), labs)


@pytest.mark.parametrize("n,m,dens", [(0, 3, 0.0), (9, 7, 0.5), (4000, 2652, 0.003), (3000, 257, 0.2)])
def test_load_and_serialize(oracle_mod, n, m, dens):
    """BinRelWT_sdsl::load / serialize (bin_rel_wt_sdsl.cpp:113-132): a stream
    written from CSR loads into a device matrix that answers like the oracle,
    and the device matrix serialises back to the same bytes (byte layout
    parity unpinned: sdsl absent)."""
    from genome_graph_annotation_amd import BinRelWTDevice
    from genome_graph_annotation_amd.binrel_wt import serialize_csr
    O = oracle_mod
    rng = np.random.default_rng(n + 7 * m)
    dense = rng.random((n, m)) < dens
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(dense.sum(1), out=off[1:])
    cols = np.nonzero(dense)[1].astype(np.uint32)
    data = serialize_csr(off, cols, m)
    d = BinRelWTDevice.load(data)
    if n:
        _compare(O, O.OracleWT.from_dense(dense), d, cols=range(min(m, 40)))
    assert d.serialize() == data
