"""Python mirror of BinRelWT_sdsl (annotation/bin_rel_wt/bin_rel_wt_sdsl.hpp)
over the device wavelet-matrix engine (include/mbrwt_wt.h).

The C++ mirror for C++ callers is csrc/binrel_wt_device.hpp; this module is
what the Python tests and tools/bench_binrel_wt.py drive.  Device-buffer
entry points take torch tensors only as plumbing for device memory/streams.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def _bytes_call(fn, what):
    """Capacity protocol for a byte stream: size, then fill."""
    need = C.c_uint64(0)
    rc = fn(None, 0, C.byref(need))
    if rc not in (L.MBRWT_OK, L.MBRWT_ERR_CAPACITY):
        L.check(rc, what)
    buf = (C.c_uint8 * max(1, need.value))()
    L.check(fn(buf, need.value, C.byref(need)), what)
    return bytes(buf[: need.value])


def _binrel_desc(offsets, cols, num_columns):
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    cols = np.ascontiguousarray(cols, dtype=np.uint32)
    if not cols.size:
        cols = np.zeros(1, dtype=np.uint32)
    d = L.BinRelDesc()
    d.num_rows = len(offsets) - 1
    d.num_columns = int(num_columns)
    d.offsets = _p(offsets, C.c_uint64)
    d.cols = _p(cols, C.c_uint32)
    return d, (offsets, cols)


def serialize_csr(offsets, cols, num_columns) -> bytes:
    """BinRelWT_sdsl::serialize (bin_rel_wt_sdsl.cpp:124-132) of CSR rows, host
    only (mbrwt_wt_serialize_desc; byte layout parity unpinned)."""
    d, keep = _binrel_desc(offsets, cols, num_columns)
    return _bytes_call(lambda b, c, n: L.lib().mbrwt_wt_serialize_desc(C.byref(d), b, c, n),
                       "mbrwt_wt_serialize_desc")


def parse_stream(data: bytes):
    """BinRelWT_sdsl::load (bin_rel_wt_sdsl.cpp:113-122) into CSR, host only:
    (offsets, cols, num_columns, bytes consumed)."""
    buf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    h = C.c_void_p()
    used = C.c_uint64(0)
    L.check(L.lib().mbrwt_wt_parse(buf, len(data), C.byref(used), C.byref(h)), "mbrwt_wt_parse")
    try:
        d = L.lib().mbrwt_binrel_get_desc(h).contents
        n = d.num_rows
        off = np.ctypeslib.as_array(d.offsets, shape=(n + 1,)).copy()
        nrel = int(off[-1])
        cols = np.ctypeslib.as_array(d.cols, shape=(nrel,)).copy() if nrel else np.zeros(0, dtype=np.uint32)
        return off, cols, int(d.num_columns), int(used.value)
    finally:
        L.lib().mbrwt_binrel_free(h)


class BinRelWTDevice:
    """A BinRel-WT held in HBM; queries run the HIP wavelet-matrix kernels."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def from_csr(cls, offsets, cols, num_columns, device=0):
        """Rows as CSR (offsets[num_rows+1], cols): the rows generate_rows
        would emit (bin_rel_wt_sdsl.cpp:10-40)."""
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        cols = np.ascontiguousarray(cols, dtype=np.uint32)
        d = L.BinRelDesc()
        d.num_rows = len(offsets) - 1
        d.num_columns = int(num_columns)
        d.offsets = _p(offsets, C.c_uint64)
        d.cols = _p(cols if cols.size else np.zeros(1, dtype=np.uint32), C.c_uint32)
        h = C.c_void_p()
        L.check(L.lib().mbrwt_wt_create(C.byref(d), device, C.byref(h)), "mbrwt_wt_create")
        return cls(h)

    @classmethod
    def from_dense(cls, dense, device=0):
        dense = np.asarray(dense, dtype=bool)
        counts = dense.sum(axis=1).astype(np.uint64)
        offsets = np.zeros(dense.shape[0] + 1, dtype=np.uint64)
        np.cumsum(counts, out=offsets[1:])
        return cls.from_csr(offsets, np.nonzero(dense)[1].astype(np.uint32), dense.shape[1], device)

    @classmethod
    def synthetic(cls, num_rows, num_columns, density, seed=42, device=0):
        d = L.BinRelSynthDesc()
        d.num_rows = int(num_rows)
        d.num_columns = int(num_columns)
        d.density = float(density)
        d.seed = int(seed)
        h = C.c_void_p()
        L.check(L.lib().mbrwt_wt_create_synthetic(C.byref(d), device, C.byref(h)), "mbrwt_wt_create_synthetic")
        return cls(h)

    @classmethod
    def load(cls, data: bytes, device=0):
        """BinRelWT_sdsl::load (bin_rel_wt_sdsl.cpp:113-122): mbrwt_wt_load."""
        buf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
        h = C.c_void_p()
        L.check(L.lib().mbrwt_wt_load(buf, len(data), None, device, C.byref(h)), "mbrwt_wt_load")
        return cls(h)

    def serialize(self) -> bytes:
        """BinRelWT_sdsl::serialize (bin_rel_wt_sdsl.cpp:124-132): mbrwt_wt_serialize."""
        return _bytes_call(lambda b, c, n: L.lib().mbrwt_wt_serialize(self._h, b, c, n), "mbrwt_wt_serialize")

    def __del__(self):
        if getattr(self, "_h", None):
            L.lib().mbrwt_wt_destroy(self._h)
            self._h = None

    def num_rows(self):
        return L.lib().mbrwt_wt_num_rows(self._h)

    def num_columns(self):
        return L.lib().mbrwt_wt_num_columns(self._h)

    def num_relations(self):
        return L.lib().mbrwt_wt_num_relations(self._h)

    def device_bytes(self):
        return L.lib().mbrwt_wt_device_bytes(self._h)

    def get_rows(self, rows):
        """Batched get_row (bin_rel_wt_sdsl.cpp:51-83) -> CSR (offsets, cols)."""
        rows = np.ascontiguousarray(rows, dtype=np.uint64)
        n = len(rows)
        offsets = np.zeros(n + 1, dtype=np.uint64)
        need = C.c_uint64(0)
        rp = _p(rows if n else np.zeros(1, dtype=np.uint64), C.c_uint64)
        st = L.lib().mbrwt_wt_get_rows(self._h, rp, n, _p(offsets, C.c_uint64), None, 0, C.byref(need))
        if st != L.MBRWT_ERR_CAPACITY:
            L.check(st, "mbrwt_wt_get_rows")
            return offsets, np.zeros(0, dtype=np.uint32)
        cols = np.zeros(max(1, need.value), dtype=np.uint32)
        L.check(L.lib().mbrwt_wt_get_rows(self._h, rp, n, _p(offsets, C.c_uint64), _p(cols, C.c_uint32), len(cols),
                                          C.byref(need)), "mbrwt_wt_get_rows")
        return offsets, cols[: need.value]

    def get_row(self, row):
        off, cols = self.get_rows([row])
        return cols.tolist()

    def get_batch(self, rows, cols):
        """Batched get (bin_rel_wt_sdsl.cpp:98-109)."""
        rows = np.ascontiguousarray(rows, dtype=np.uint64)
        cols = np.ascontiguousarray(cols, dtype=np.uint64)
        out = np.zeros(max(1, len(rows)), dtype=np.uint8)
        L.check(L.lib().mbrwt_wt_get_batch(self._h, _p(rows, C.c_uint64), _p(cols, C.c_uint64), len(rows),
                                           _p(out, C.c_uint8)), "mbrwt_wt_get_batch")
        return out[: len(rows)].astype(bool)

    def get(self, row, col):
        return bool(self.get_batch([row], [col])[0])

    def get_column(self, col):
        """get_column (bin_rel_wt_sdsl.cpp:85-96): ascending rows."""
        need = C.c_uint64(0)
        st = L.lib().mbrwt_wt_get_column(self._h, int(col), None, 0, C.byref(need))
        if st != L.MBRWT_ERR_CAPACITY:
            L.check(st, "mbrwt_wt_get_column")
            return np.zeros(0, dtype=np.uint64)
        out = np.zeros(max(1, need.value), dtype=np.uint64)
        L.check(L.lib().mbrwt_wt_get_column(self._h, int(col), _p(out, C.c_uint64), len(out), C.byref(need)),
                "mbrwt_wt_get_column")
        return out[: need.value]

    # -- device buffers --------------------------------------------------------
    def get_rows_device(self, rows_t, offsets_t, cols_t, stream=None):
        need = C.c_uint64(0)
        st = L.lib().mbrwt_wt_get_rows_device(self._h, rows_t.data_ptr(), rows_t.numel(), offsets_t.data_ptr(),
                                              cols_t.data_ptr(), cols_t.numel(), C.byref(need), stream)
        if st == L.MBRWT_ERR_CAPACITY:
            e = L.MBRWTError(st, "mbrwt_wt_get_rows_device")
            e.needed = int(need.value)
            raise e
        L.check(st, "mbrwt_wt_get_rows_device")
        return int(need.value)

    # -- batched classify (include/mbrwt_wt.h; semantics as BRWTDevice's) ------
    def get_labels_batch(self, rows, read_offsets, presence_ratio):
        from .brwt import _labels_batch
        return _labels_batch("mbrwt_wt_get_labels_batch", self._h, rows, read_offsets, presence_ratio)

    def get_top_labels_batch(self, rows, read_offsets, num_top=2**64 - 1):
        from .brwt import _top_labels_batch
        return _top_labels_batch("mbrwt_wt_get_top_labels_batch", self._h, rows, read_offsets, num_top)

    def get_labels_batch_device(self, rows_t, read_off_t, presence_ratio, lab_off_t, labels_t, stream=None):
        need = C.c_uint64(0)
        st = L.lib().mbrwt_wt_get_labels_batch_device(
            self._h, rows_t.data_ptr(), rows_t.numel(), read_off_t.data_ptr(), read_off_t.numel() - 1,
            float(presence_ratio), lab_off_t.data_ptr(), labels_t.data_ptr() if labels_t is not None else None,
            labels_t.numel() if labels_t is not None else 0, C.byref(need), stream)
        if st == L.MBRWT_ERR_CAPACITY:
            e = L.MBRWTError(st, "mbrwt_wt_get_labels_batch_device")
            e.needed = int(need.value)
            raise e
        L.check(st, "mbrwt_wt_get_labels_batch_device")
        return int(need.value)

    def set_option(self, option, value):
        L.check(L.lib().mbrwt_wt_set_option(self._h, option, int(value)), "mbrwt_wt_set_option")

    def take_timing(self):
        ms = C.c_double(0)
        k = C.c_uint64(0)
        L.check(L.lib().mbrwt_wt_take_timing(self._h, C.byref(ms), C.byref(k)), "mbrwt_wt_take_timing")
        return ms.value, int(k.value)
