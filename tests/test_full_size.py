"""Full-size parity of the named single-GPU configurations (BASELINE.json
configs[2] and [4]) -- the structures at their full row counts, the full query
batch, every label checked element-wise (and a 64-bit hash of the CSR, the
SURVEY §8(d) parity gate).

* C3: Multi-BRWT 1,000,000,000 x 3,173, d = 3.8 %, arity 8 (RefSeq shape),
  10,000,000 uniform random rows (seed 42).  The oracle side does not build
  the 158 GB of plain index bits on the host: oracle.topdown_get_rows streams
  the same synthetic tree (every index bit is a pure function of node and
  position) and restates BRWT::get_row (BRWT.cpp:26-53) with exact inclusive
  ranks; it is checked against the materialised oracle tree in
  tests/test_oracle_stream.py.
* C4: the 3.7 B x 2,652 Kingsford-shaped Multi-BRWT (BASELINE configs[3],
  the bench's structure) as row records (the bench's layout), against the
  same streamed oracle.
* C5: BinRel-WT(sdsl) 1,000,000,000 x 3,173, d = 3.8 %, 10,000,000 rows
  (seed 43): the rows of the synthetic matrix are row-independent (a counter
  hash per cell), so the oracle evaluates exactly the queried rows; the
  BinRel-WT restatement itself (bin_rel_wt_sdsl.cpp:51-83) is pinned against
  the same generator in tests/test_gpu_binrel_wt.py.

Host memory: about 30 GB (C3: the CSR on both sides plus the oracle's
emission list).  Device memory: 214 GB (C3) and 231 GB (C5), one at a time.
"""
import hashlib
import os
import time

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.slow,
              pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def _threads():
    share = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return min(share, omp) if omp > 0 else share


def _hash(off, cols):
    h = hashlib.blake2b(digest_size=8)
    h.update(np.ascontiguousarray(off, dtype=np.uint64).tobytes())
    h.update(np.ascontiguousarray(cols, dtype=np.uint32).tobytes())
    return h.hexdigest()


def _release():
    import gc

    import torch
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


@pytest.mark.timeout(900)
def test_c3_refseq_multibrwt_full_size(oracle_mod):
    from genome_graph_annotation_amd import BRWTDevice

    n, m, d, arity, batch = 1_000_000_000, 3173, 0.038, 8, 10_000_000
    t0 = time.time()
    dev = BRWTDevice.synthetic(n, m, d, arity, 42)
    build_s = time.time() - t0
    rows = np.random.default_rng(42).integers(0, n, batch, dtype=np.uint64)
    try:
        off_d, cols_d = dev.get_rows(rows)
        dev_bytes = dev.device_bytes()
    finally:
        dev.close()
        _release()
    t0 = time.time()
    off_o, cols_o, draws = oracle_mod.topdown_get_rows(n, m, d, arity, 42, rows, _threads(), with_draws=True)
    oracle_s = time.time() - t0
    print(f"C3 {n:,} x {m:,}: device {dev_bytes / 1e9:.1f} GB built in {build_s:.1f} s; "
          f"{len(cols_d):,} labels for {batch:,} rows; oracle streamed {draws:,} draws in {oracle_s:.0f} s "
          f"on {_threads()} threads; CSR hash device {_hash(off_d, cols_d)} oracle {_hash(off_o, cols_o)}")
    assert np.array_equal(off_d, off_o)
    assert np.array_equal(cols_d, cols_o)
    assert 115 < len(cols_o) / batch < 126  # E[L] = 120.6 labels per row at this shape


@pytest.mark.timeout(900)
def test_c4_kingsford_rows_full_size(oracle_mod):
    """BASELINE configs[3]'s structure on one GPU in the bench's layout: the
    3.7 B x 2,652 Kingsford-shaped Multi-BRWT (d = 0.3 %, arity 8) as row
    records, against the streamed oracle -- 2 M uniform random rows, the first
    and last rows, the rows around every range boundary of the ranged build
    and around 2^31 / 2^32, then the 16,384 rows of the first 4 M with the
    most labels (long records: spilled entries and direct tiles) as a batch
    of their own."""
    from genome_graph_annotation_amd import BRWTDevice

    n, m, d, arity = 3_700_000_000, 2652, 0.003, 8
    t0 = time.time()
    dev = BRWTDevice.synthetic(n, m, d, arity, 42, layout="rows")
    build_s = time.time() - t0
    rng = np.random.default_rng(44)
    edges = [0, n - 1]
    rng_rows = 2979 * 360360  # rows per range of the ranged build (capi.cpp rows_range_rows)
    for e in list(range(rng_rows, n, rng_rows)) + [2**31, 2**32 - 1]:
        edges += list(range(e - 8, min(e + 8, n)))
    rows = np.concatenate([np.array(edges, dtype=np.uint64), rng.integers(0, n, 2_000_000, dtype=np.uint64)])
    pool = rng.integers(0, n, 4_000_000, dtype=np.uint64)
    try:
        st = dev.rows_stats()
        assert dev.layout() == "rows" and st["uniform_levels"] == 3
        off_d, cols_d = dev.get_rows(rows)
        off_p, _ = dev.get_rows(pool)
        longest = pool[np.argsort(np.diff(off_p.astype(np.int64)), kind="stable")[-16384:]]
        off_l, cols_l = dev.get_rows(longest)
        dev_bytes = dev.device_bytes()
    finally:
        dev.close()
        _release()
    t0 = time.time()
    off_o, cols_o = oracle_mod.topdown_get_rows(n, m, d, arity, 42, rows, _threads())
    off_lo, cols_lo = oracle_mod.topdown_get_rows(n, m, d, arity, 42, longest, _threads())
    oracle_s = time.time() - t0
    print(f"C4 {n:,} x {m:,} rows layout: {dev_bytes / 1e9:.1f} GB built in {build_s:.1f} s "
          f"(B={st['block_bytes']}, S={st['rows_per_block']}, {st['spilled_rows']:,} spilled, "
          f"{st['long_rows']:,} long); {len(cols_d):,} labels for {len(rows):,} rows; long batch "
          f"{len(cols_l):,} labels ({np.diff(off_l.astype(np.int64)).min()}+ per row); oracle {oracle_s:.0f} s; "
          f"CSR hash device {_hash(off_d, cols_d)} oracle {_hash(off_o, cols_o)}")
    assert np.array_equal(off_d, off_o)
    assert np.array_equal(cols_d, cols_o)
    assert np.array_equal(off_l, off_lo)
    assert np.array_equal(cols_l, cols_lo)
    assert 7.5 < len(cols_o) / len(rows) < 8.5  # E[L] = 7.96 labels per row at this shape


@pytest.mark.timeout(900)
def test_c5_refseq_binrel_wt_full_size(oracle_mod):
    from genome_graph_annotation_amd import BinRelWTDevice

    n, m, d, batch = 1_000_000_000, 3173, 0.038, 10_000_000
    t0 = time.time()
    wt = BinRelWTDevice.synthetic(n, m, d, 42)
    build_s = time.time() - t0
    rows = np.random.default_rng(43).integers(0, n, batch, dtype=np.uint64)
    try:
        off_d, cols_d = wt.get_rows(rows)
        rel, dev_bytes = wt.num_relations(), wt.device_bytes()
    finally:
        del wt
        _release()
    t0 = time.time()
    off_o, cols_o = oracle_mod.wt_synth_rows_at(rows, m, d, 42, _threads())
    oracle_s = time.time() - t0
    print(f"C5 {n:,} x {m:,}: {rel:,} relations, {dev_bytes / 1e9:.1f} GB built in {build_s:.1f} s; "
          f"{len(cols_d):,} labels for {batch:,} rows; oracle {oracle_s:.0f} s; "
          f"CSR hash device {_hash(off_d, cols_d)} oracle {_hash(off_o, cols_o)}")
    assert np.array_equal(off_d, off_o)
    assert np.array_equal(cols_d, cols_o)
