"""ctypes wrapper of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  It is the checker for the HIP product path
(genome_graph_annotation_amd), never part of it.  See brwt_oracle.h for the
reference file:line each entry point restates.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

u64p = C.POINTER(C.c_uint64)
u32p = C.POINTER(C.c_uint32)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        build()
    L = C.CDLL(_LIB_PATH)
    vp = C.c_void_p
    sig = {
        "oracle_build_from_columns": (vp, [u64p, C.c_uint64, C.c_uint64, C.c_int, C.c_uint32, C.c_uint64]),
        "oracle_generate_norepl": (vp, [C.c_uint64, C.c_uint64, C.c_double, C.c_uint32, C.c_int, C.c_uint32, C.c_uint64]),
        "oracle_generate_uniform_rows": (C.c_uint64, [C.c_uint64, C.c_uint64, C.c_double, C.c_uint64, C.c_uint32, vp]),
        "oracle_generate_uniform_columns": (C.c_uint64, [C.c_uint64, C.c_uint64, C.c_double, C.c_uint64, C.c_uint32, vp]),
        "oracle_rrr_bytes": (C.c_uint64, [vp]),
        "oracle_generate_topdown": (vp, [C.c_uint64, C.c_uint64, C.c_double, C.c_uint32, C.c_uint64, C.c_int]),
        "oracle_free": (None, [vp]),
        "oracle_num_rows": (C.c_uint64, [vp]),
        "oracle_num_columns": (C.c_uint64, [vp]),
        "oracle_num_relations": (C.c_uint64, [vp]),
        "oracle_num_nodes": (C.c_uint64, [vp]),
        "oracle_avg_arity": (C.c_double, [vp]),
        "oracle_total_column_size": (C.c_uint64, [vp]),
        "oracle_total_num_set_bits": (C.c_uint64, [vp]),
        "oracle_depth": (C.c_uint32, [vp]),
        "oracle_get": (C.c_int, [vp, C.c_uint64, C.c_uint64]),
        "oracle_get_row": (C.c_uint64, [vp, C.c_uint64, u32p, C.c_uint64, u64p]),
        "oracle_get_rows": (C.c_int, [vp, u64p, C.c_uint64, u64p, u32p, C.c_uint64, u64p, u32p, C.c_int]),
        "oracle_time_rows": (C.c_uint64, [vp, u64p, C.c_uint64, C.c_int]),
        "oracle_get_column": (C.c_uint64, [vp, C.c_uint64, u64p, C.c_uint64]),
        "oracle_export_num_nodes": (C.c_uint32, [vp]),
        "oracle_export": (None, [vp, u32p, u32p, u32p, u64p]),
        "oracle_export_vec_words": (u64p, [vp, C.c_uint32]),
        "oracle_generate_random_ints": (None, [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, u64p]),
        "oracle_generate_columns": (None, [C.c_uint64, C.c_uint64, C.c_double, C.c_uint32, u64p]),
        "oracle_bv_new": (vp, [u64p, C.c_uint64]),
        "oracle_bv_free": (None, [vp]),
        "oracle_bv_rank1": (C.c_uint64, [vp, C.c_uint64]),
        "oracle_bv_select1": (C.c_uint64, [vp, C.c_uint64]),
        "oracle_bv_get": (C.c_int, [vp, C.c_uint64]),
        "oracle_bv_num_set_bits": (C.c_uint64, [vp]),
        "oracle_synth_hash": (C.c_uint64, [C.c_uint64, C.c_uint64, C.c_uint64]),
        # BinRel-WT(sdsl) restatement (binrel_wt_oracle.h)
        "wt_oracle_build": (vp, [u64p, u32p, C.c_uint64, C.c_uint64]),
        "wt_oracle_empty": (vp, []),
        "wt_oracle_free": (None, [vp]),
        "wt_oracle_num_rows": (C.c_uint64, [vp]),
        "wt_oracle_num_columns": (C.c_uint64, [vp]),
        "wt_oracle_num_relations": (C.c_uint64, [vp]),
        "wt_oracle_get_row": (C.c_uint64, [vp, C.c_uint64, u32p, C.c_uint64]),
        "wt_oracle_get": (C.c_int, [vp, C.c_uint64, C.c_uint64]),
        "wt_oracle_get_column": (C.c_uint64, [vp, C.c_uint64, u64p, C.c_uint64]),
        "wt_oracle_get_rows": (C.c_int, [vp, u64p, C.c_uint64, u64p, u32p, C.c_uint64, u64p, C.c_int]),
        "wt_oracle_time_rows": (C.c_double, [vp, u64p, C.c_uint64, C.c_int]),
        "wt_synth_threshold": (C.c_uint64, [C.c_double]),
        "wt_synth_row": (C.c_uint64, [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, u32p, C.c_uint64]),
        "wt_synth_rows": (C.c_int, [C.c_uint64, C.c_uint64, C.c_uint64, C.c_double, C.c_uint64, u64p, u32p,
                                    C.c_uint64, u64p, C.c_int]),
        "wt_synth_rows_at": (C.c_int, [u64p, C.c_uint64, C.c_uint64, C.c_double, C.c_uint64, u64p, u32p,
                                       C.c_uint64, u64p, C.c_int]),
        "oracle_topdown_get_rows": (vp, [C.c_uint64, C.c_uint64, C.c_double, C.c_uint32, C.c_uint64, u64p,
                                         C.c_uint64, C.c_int, C.POINTER(C.c_int)]),
        "oracle_csr_num_labels": (C.c_uint64, [vp]),
        "oracle_csr_draws": (C.c_uint64, [vp]),
        "oracle_csr_copy": (None, [vp, u64p, u32p]),
        "oracle_csr_free": (None, [vp]),
        "oracle_to_rrr": (None, [vp, C.c_int]),
        "oracle_topdown_get_rows_shaped": (vp, [C.c_uint64, C.c_uint32, u32p, u32p, u32p, C.c_double, C.c_uint64,
                                                u64p, C.c_uint64, C.c_int, C.POINTER(C.c_int)]),
        "oracle_generate_topdown_shaped": (vp, [C.c_uint64, C.c_uint32, u32p, u32p, u32p, C.c_double, C.c_uint64,
                                                C.c_int]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _p64(a):
    return a.ctypes.data_as(u64p)


def _p32(a):
    return a.ctypes.data_as(u32p)


def pack_columns(dense: np.ndarray) -> np.ndarray:
    """dense bool matrix [rows, cols] -> column-major LSB-first u64 words."""
    dense = np.asarray(dense, dtype=bool)
    n, m = dense.shape
    W = (n + 63) // 64
    out = np.zeros((m, W * 64), dtype=bool)
    out[:, :n] = dense.T
    return np.packbits(out.reshape(m, W, 64), axis=2, bitorder="little").view(np.uint64).reshape(m * W).copy()


class BitVec:
    """bit_vector rank/select/access semantics (common/bit_vector.hpp:12-45)."""

    def __init__(self, bits):
        bits = np.asarray(bits, dtype=bool)
        self.size = len(bits)
        W = max(1, (self.size + 63) // 64)
        pad = np.zeros(W * 64, dtype=bool)
        pad[: self.size] = bits
        self._words = np.packbits(pad.reshape(W, 64), axis=1, bitorder="little").view(np.uint64).reshape(W).copy()
        self._h = lib().oracle_bv_new(_p64(self._words), self.size)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().oracle_bv_free(self._h)
            self._h = None

    def rank1(self, i):
        return lib().oracle_bv_rank1(self._h, i)

    def select1(self, i):
        r = lib().oracle_bv_select1(self._h, i)
        if r == 2**64 - 1:
            raise IndexError("select1 out of range")
        return r

    def __getitem__(self, i):
        r = lib().oracle_bv_get(self._h, i)
        if r < 0:
            raise IndexError(i)
        return r

    def num_set_bits(self):
        return lib().oracle_bv_num_set_bits(self._h)


class OracleTree:
    """A BRWT held by the oracle (the reference's BRWT semantics)."""

    def __init__(self, handle):
        if not handle:
            raise RuntimeError("oracle construction failed")
        self._h = handle

    def __del__(self):
        if getattr(self, "_h", None):
            lib().oracle_free(self._h)
            self._h = None

    # -- constructors --------------------------------------------------------
    @classmethod
    def from_dense(cls, dense, partitioner="basic", arity=2, relax=0):
        dense = np.asarray(dense, dtype=bool)
        n, m = dense.shape if dense.ndim == 2 else (0, 0)
        words = pack_columns(dense) if m else np.zeros(1, dtype=np.uint64)
        p = {"basic": 0, "greedy": 1}[partitioner]
        return cls(lib().oracle_build_from_columns(_p64(words), n, m, p, arity, relax))

    @classmethod
    def from_words(cls, words, n, m, partitioner="basic", arity=2, relax=0):
        """From column-major packed words (generate_columns and friends)."""
        p = {"basic": 0, "greedy": 1}[partitioner]
        return cls(lib().oracle_build_from_columns(_p64(words), n, m, p, arity, relax))

    @classmethod
    def norepl(cls, n, m, d, seed=42, partitioner="basic", arity=2, relax=0):
        p = {"basic": 0, "greedy": 1}[partitioner]
        return cls(lib().oracle_generate_norepl(n, m, d, seed, p, arity, relax))

    @classmethod
    def topdown(cls, n, m, d, arity=8, seed=42, threads=0):
        return cls(lib().oracle_generate_topdown(n, m, d, arity, seed, threads))

    @classmethod
    def topdown_shaped(cls, n, shape, d, seed=42, threads=0):
        """The top-down law over a given shape (dict with num_children,
        first_child, leaf_column in BFS order, e.g. another tree's export)."""
        nc, fc, lc = _shape_arrays(shape)
        return cls(lib().oracle_generate_topdown_shaped(n, len(nc), _p32(nc), _p32(fc), _p32(lc), d, seed, threads))

    # -- BinaryMatrix surface -------------------------------------------------
    def num_rows(self):
        return lib().oracle_num_rows(self._h)

    def num_columns(self):
        return lib().oracle_num_columns(self._h)

    def num_relations(self):
        return lib().oracle_num_relations(self._h)

    def num_nodes(self):
        return lib().oracle_num_nodes(self._h)

    def avg_arity(self):
        return lib().oracle_avg_arity(self._h)

    def depth(self):
        return lib().oracle_depth(self._h)

    def total_column_size(self):
        return lib().oracle_total_column_size(self._h)

    def total_num_set_bits(self):
        return lib().oracle_total_num_set_bits(self._h)

    def get(self, row, col):
        r = lib().oracle_get(self._h, row, col)
        if r < 0:
            raise IndexError((row, col))
        return bool(r)

    def get_row(self, row, with_visits=False):
        cap = max(1, self.num_columns())
        out = np.zeros(cap, dtype=np.uint32)
        v = C.c_uint64(0)
        cnt = lib().oracle_get_row(self._h, row, _p32(out), cap, C.byref(v))
        if cnt == 2**64 - 1:
            raise IndexError(row)
        res = out[:cnt].tolist()
        return (res, v.value) if with_visits else res

    def get_rows(self, rows, threads=0, with_visits=False):
        rows = np.ascontiguousarray(rows, dtype=np.uint64)
        n = len(rows)
        offsets = np.zeros(n + 1, dtype=np.uint64)
        visits = np.zeros(max(1, n), dtype=np.uint32)
        need = C.c_uint64(0)
        dummy = np.zeros(1, dtype=np.uint32)
        rc = lib().oracle_get_rows(self._h, _p64(rows), n, _p64(offsets), _p32(dummy), 0, C.byref(need), _p32(visits), threads)
        if rc == 2:
            raise IndexError("row out of range")
        cols = np.zeros(max(1, need.value), dtype=np.uint32)
        rc = lib().oracle_get_rows(self._h, _p64(rows), n, _p64(offsets), _p32(cols), len(cols), C.byref(need), _p32(visits), threads)
        assert rc == 0
        cols = cols[: need.value]
        return (offsets, cols, visits[:n]) if with_visits else (offsets, cols)

    def time_rows(self, rows, threads=0):
        rows = np.ascontiguousarray(rows, dtype=np.uint64)
        return lib().oracle_time_rows(self._h, _p64(rows), len(rows), threads)

    def rrr_bytes(self):
        """Bytes of every node's index as an sdsl rrr_vector<63> stream."""
        return lib().oracle_rrr_bytes(self._h)

    def to_rrr(self, threads=0):
        """Re-encode the indexes sdsl-RRR-like (CPU baseline); afterwards
        only get / get_row(s) / time_rows are valid."""
        lib().oracle_to_rrr(self._h, threads)
        return self

    def get_column(self, col):
        cap = max(1, self.num_rows())
        out = np.zeros(cap, dtype=np.uint64)
        cnt = lib().oracle_get_column(self._h, col, _p64(out), cap)
        if cnt == 2**64 - 1:
            raise IndexError(col)
        return out[:cnt].tolist()

    # -- BFS export (the tree description of include/mbrwt.h) ----------------
    def export(self):
        """Returns dict with num_children, first_child, leaf_column, vec_size
        (numpy arrays, BFS numbering) and `words`: list of u64 arrays."""
        L = lib()
        N = L.oracle_export_num_nodes(self._h)
        nc = np.zeros(max(1, N), dtype=np.uint32)
        fc = np.zeros(max(1, N), dtype=np.uint32)
        lc = np.zeros(max(1, N), dtype=np.uint32)
        vs = np.zeros(max(1, N), dtype=np.uint64)
        if N:
            L.oracle_export(self._h, _p32(nc), _p32(fc), _p32(lc), _p64(vs))
        words = []
        for u in range(N):
            W = (int(vs[u]) + 63) // 64
            p = L.oracle_export_vec_words(self._h, u)
            if W:
                words.append(np.ctypeslib.as_array(p, shape=(W,)).copy())
            else:
                words.append(np.zeros(0, dtype=np.uint64))
        return dict(num_nodes=N, num_rows=self.num_rows(), num_columns=self.num_columns(),
                    num_children=nc[:N], first_child=fc[:N], leaf_column=lc[:N], vec_size=vs[:N], words=words)


def generate_random_ints(n, begin, end, seed=42):
    """experiments/data_generation.cpp:7-18 (std::uniform_int_distribution<int>)."""
    out = np.zeros(max(1, n), dtype=np.uint64)
    lib().oracle_generate_random_ints(n, begin, end, seed, _p64(out))
    return out[:n]


def generate_uniform_rows(n, m, d, unique, seed=42):
    """experiments/main.cpp "uniform_rows": (column-major words, rows)."""
    rows = (n // unique) * unique
    W = (rows + 63) // 64
    out = np.zeros(max(1, W * m), dtype=np.uint64)
    got = lib().oracle_generate_uniform_rows(n, m, d, unique, seed, out.ctypes.data)
    assert got == rows
    return out, rows


def generate_uniform_columns(n, m, d, unique, seed=42):
    """experiments/main.cpp "uniform_columns": (column-major words, columns)."""
    cols = (m // unique) * unique
    W = (n + 63) // 64
    out = np.zeros(max(1, W * cols), dtype=np.uint64)
    got = lib().oracle_generate_uniform_columns(n, m, d, unique, seed, out.ctypes.data)
    assert got == cols
    return out, cols


def generate_columns(n, m, d, seed=42):
    W = (n + 63) // 64
    out = np.zeros(max(1, W * m), dtype=np.uint64)
    lib().oracle_generate_columns(n, m, d, seed, _p64(out))
    return out


def synth_hash(seed, key, pos):
    return lib().oracle_synth_hash(seed, key, pos)


def _shape_arrays(shape):
    return (np.ascontiguousarray(shape["num_children"], dtype=np.uint32),
            np.ascontiguousarray(shape["first_child"], dtype=np.uint32),
            np.ascontiguousarray(shape["leaf_column"], dtype=np.uint32))


def _csr_out(h, n):
    try:
        nl = lib().oracle_csr_num_labels(h)
        off = np.zeros(n + 1, dtype=np.uint64)
        cols = np.zeros(max(1, nl), dtype=np.uint32)
        lib().oracle_csr_copy(h, _p64(off), _p32(cols))
        draws = lib().oracle_csr_draws(h)
    finally:
        lib().oracle_csr_free(h)
    return off, cols[:nl], draws


def topdown_get_rows_shaped(n, shape, d, seed, rows, threads=0):
    """topdown_get_rows over a given shape (see OracleTree.topdown_shaped)."""
    rows = np.ascontiguousarray(rows, dtype=np.uint64)
    nc, fc, lc = _shape_arrays(shape)
    st = C.c_int(0)
    h = lib().oracle_topdown_get_rows_shaped(n, len(nc), _p32(nc), _p32(fc), _p32(lc), d, seed, _p64(rows),
                                             len(rows), threads, C.byref(st))
    if st.value == 2:
        raise IndexError("row out of range")
    if st.value:
        raise ValueError("malformed shape")
    off, cols, _ = _csr_out(h, len(rows))
    return off, cols


def topdown_get_rows(n, m, d, arity, seed, rows, threads=0, with_draws=False):
    """BRWT::get_row over the top-down synthetic tree (n x m, density d) for
    rows[], streamed without building the tree (brwt_oracle.h)."""
    rows = np.ascontiguousarray(rows, dtype=np.uint64)
    st = C.c_int(0)
    h = lib().oracle_topdown_get_rows(n, m, d, arity, seed, _p64(rows), len(rows), threads, C.byref(st))
    if st.value == 2:
        raise IndexError("row out of range")
    try:
        nl = lib().oracle_csr_num_labels(h)
        off = np.zeros(len(rows) + 1, dtype=np.uint64)
        cols = np.zeros(max(1, nl), dtype=np.uint32)
        lib().oracle_csr_copy(h, _p64(off), _p32(cols))
        draws = lib().oracle_csr_draws(h)
    finally:
        lib().oracle_csr_free(h)
    return (off, cols[:nl], draws) if with_draws else (off, cols[:nl])


# ---- BinRel-WT(sdsl) (binrel_wt_oracle.h) ------------------------------------

def dense_to_csr(dense: np.ndarray):
    """rows of a dense bool matrix -> CSR (offsets u64, cols u32), ascending ids"""
    dense = np.asarray(dense, dtype=bool)
    counts = dense.sum(axis=1).astype(np.uint64)
    offsets = np.zeros(dense.shape[0] + 1, dtype=np.uint64)
    np.cumsum(counts, out=offsets[1:])
    cols = np.nonzero(dense)[1].astype(np.uint32)
    return offsets, cols


def wt_synth_rows(row0, n, num_columns, density, seed=42, threads=0):
    """CSR of synthetic BinRel rows [row0, row0+n) (DESIGN.md "BinRel-WT")."""
    offsets = np.zeros(n + 1, dtype=np.uint64)
    need = C.c_uint64(0)
    dummy = np.zeros(1, dtype=np.uint32)
    lib().wt_synth_rows(row0, n, num_columns, density, seed, _p64(offsets), _p32(dummy), 0, C.byref(need), threads)
    cols = np.zeros(max(1, need.value), dtype=np.uint32)
    rc = lib().wt_synth_rows(row0, n, num_columns, density, seed, _p64(offsets), _p32(cols), len(cols),
                             C.byref(need), threads)
    assert rc == 0
    return offsets, cols[: need.value]


def wt_synth_rows_at(rows, num_columns, density, seed=42, threads=0):
    """CSR of the synthetic BinRel rows rows[] (any order, repeats allowed)."""
    rows = np.ascontiguousarray(rows, dtype=np.uint64)
    n = len(rows)
    offsets = np.zeros(n + 1, dtype=np.uint64)
    need = C.c_uint64(0)
    dummy = np.zeros(1, dtype=np.uint32)
    lib().wt_synth_rows_at(_p64(rows), n, num_columns, density, seed, _p64(offsets), _p32(dummy), 0,
                           C.byref(need), threads)
    cols = np.zeros(max(1, need.value), dtype=np.uint32)
    rc = lib().wt_synth_rows_at(_p64(rows), n, num_columns, density, seed, _p64(offsets), _p32(cols), len(cols),
                                C.byref(need), threads)
    assert rc == 0
    return offsets, cols[: need.value]


class OracleWT:
    """BinRelWT_sdsl restated (annotation/bin_rel_wt/bin_rel_wt_sdsl.cpp)."""

    def __init__(self, handle):
        if not handle:
            raise ValueError("invalid BinRel-WT input")
        self._h = handle

    @classmethod
    def from_csr(cls, offsets, cols, num_columns):
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        cols = np.ascontiguousarray(cols, dtype=np.uint32)
        n = len(offsets) - 1
        cptr = cols if len(cols) else np.zeros(1, dtype=np.uint32)
        return cls(lib().wt_oracle_build(_p64(offsets), _p32(cptr), n, num_columns))

    @classmethod
    def from_dense(cls, dense):
        dense = np.asarray(dense, dtype=bool)
        off, cols = dense_to_csr(dense)
        return cls.from_csr(off, cols, dense.shape[1] if dense.ndim == 2 else 0)

    @classmethod
    def empty(cls):
        return cls(lib().wt_oracle_empty())

    def __del__(self):
        if getattr(self, "_h", None):
            lib().wt_oracle_free(self._h)
            self._h = None

    def num_rows(self):
        return lib().wt_oracle_num_rows(self._h)

    def num_columns(self):
        return lib().wt_oracle_num_columns(self._h)

    def num_relations(self):
        return lib().wt_oracle_num_relations(self._h)

    def get_row(self, row):
        buf = np.zeros(max(1, self.num_columns() + 64), dtype=np.uint32)
        cnt = lib().wt_oracle_get_row(self._h, row, _p32(buf), len(buf))
        if cnt == 2**64 - 1:
            raise IndexError(row)
        if cnt > len(buf):
            buf = np.zeros(cnt, dtype=np.uint32)
            lib().wt_oracle_get_row(self._h, row, _p32(buf), len(buf))
        return buf[:cnt].tolist()

    def get(self, row, col):
        v = lib().wt_oracle_get(self._h, row, col)
        if v < 0:
            raise IndexError((row, col))
        return bool(v)

    def get_column(self, col):
        cap = max(1, self.num_rows())
        out = np.zeros(cap, dtype=np.uint64)
        cnt = lib().wt_oracle_get_column(self._h, col, _p64(out), cap)
        if cnt == 2**64 - 1:
            raise IndexError(col)
        if cnt > cap:
            out = np.zeros(cnt, dtype=np.uint64)
            lib().wt_oracle_get_column(self._h, col, _p64(out), cnt)
        return out[:cnt]

    def get_rows(self, rows, threads=0):
        rows = np.ascontiguousarray(rows, dtype=np.uint64)
        n = len(rows)
        offsets = np.zeros(n + 1, dtype=np.uint64)
        need = C.c_uint64(0)
        dummy = np.zeros(1, dtype=np.uint32)
        rows_p = rows if n else np.zeros(1, dtype=np.uint64)
        rc = lib().wt_oracle_get_rows(self._h, _p64(rows_p), n, _p64(offsets), _p32(dummy), 0, C.byref(need), threads)
        if rc == 2:
            raise IndexError("row out of range")
        cols = np.zeros(max(1, need.value), dtype=np.uint32)
        rc = lib().wt_oracle_get_rows(self._h, _p64(rows_p), n, _p64(offsets), _p32(cols), len(cols), C.byref(need),
                                      threads)
        assert rc == 0
        return offsets, cols[: need.value]

    def time_rows(self, rows, threads=0):
        rows = np.ascontiguousarray(rows, dtype=np.uint64)
        return lib().wt_oracle_time_rows(self._h, _p64(rows), len(rows), threads)
