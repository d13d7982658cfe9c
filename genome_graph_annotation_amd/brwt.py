"""Python mirror of the reference's BinaryMatrix surface over the HIP engine.

`BRWTDevice` answers the reference's BRWT queries (BinaryMatrix,
common/binary_matrix.hpp:9-29; BRWT, annotation/hierarchical_annotation/
BRWT.hpp:33-51) from a device-resident image through include/mbrwt.h.
The C++ mirror used by C++ callers is csrc/brwt_device.hpp; this module is
what the Python tests and bench.py drive.  Device-buffer entry points take
torch tensors only as plumbing for device memory and streams.
"""
from __future__ import annotations

import contextlib
import ctypes as C

import numpy as np

from . import _lib as L


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def _labels_batch(fn, h, rows, read_offsets, presence_ratio):
    """Host-buffer batched get_labels through `fn` (mbrwt[_wt]_get_labels_batch)."""
    rows = np.ascontiguousarray(rows, dtype=np.uint64)
    ro = np.ascontiguousarray(read_offsets, dtype=np.uint64)
    if ro.size == 0:
        raise ValueError("read_offsets needs n_reads + 1 entries")
    lo = np.zeros(ro.size, dtype=np.uint64)
    need = C.c_uint64(0)
    cap = max(16, 4 * rows.size)
    while True:
        labs = np.zeros(cap, dtype=np.uint32)
        st = getattr(L.lib(), fn)(h, _p(rows, C.c_uint64), rows.size, _p(ro, C.c_uint64), ro.size - 1,
                                  float(presence_ratio), _p(lo, C.c_uint64), _p(labs, C.c_uint32), cap, C.byref(need))
        if st == L.MBRWT_ERR_CAPACITY:
            cap = int(need.value)
            continue
        L.check(st, fn)
        return lo, labs[: need.value]


def _top_labels_batch(fn, h, rows, read_offsets, num_top):
    """Host-buffer batched get_top_labels through `fn` (mbrwt[_wt]_get_top_labels_batch)."""
    rows = np.ascontiguousarray(rows, dtype=np.uint64)
    ro = np.ascontiguousarray(read_offsets, dtype=np.uint64)
    if ro.size == 0:
        raise ValueError("read_offsets needs n_reads + 1 entries")
    lo = np.zeros(ro.size, dtype=np.uint64)
    need = C.c_uint64(0)
    cap = max(16, 4 * rows.size)
    while True:
        labs = np.zeros(cap, dtype=np.uint32)
        cnts = np.zeros(cap, dtype=np.uint64)
        st = getattr(L.lib(), fn)(h, _p(rows, C.c_uint64), rows.size, _p(ro, C.c_uint64), ro.size - 1,
                                  int(num_top), _p(lo, C.c_uint64), _p(labs, C.c_uint32), _p(cnts, C.c_uint64), cap,
                                  C.byref(need))
        if st == L.MBRWT_ERR_CAPACITY:
            cap = int(need.value)
            continue
        L.check(st, fn)
        return lo, labs[: need.value], cnts[: need.value]


def tree_desc(tree):
    """mbrwt_tree_desc of a BFS tree dict (keys: num_rows, num_columns,
    num_children, first_child, leaf_column, vec_size, words); returns the
    struct and the arrays it points into (keep them alive while it is used)."""
    N = int(len(tree["num_children"]))
    nc = np.ascontiguousarray(tree["num_children"], dtype=np.uint32)
    fc = np.ascontiguousarray(tree["first_child"], dtype=np.uint32)
    lc = np.ascontiguousarray(tree["leaf_column"], dtype=np.uint32)
    vs = np.ascontiguousarray(tree["vec_size"], dtype=np.uint64)
    words = [np.ascontiguousarray(w, dtype=np.uint64) for w in tree["words"]]
    ptrs = (L.u64p * max(1, N))()
    for u, w in enumerate(words):
        ptrs[u] = _p(w, C.c_uint64) if w.size else None
    d = L.TreeDesc()
    d.num_rows = int(tree["num_rows"])
    d.num_columns = int(tree["num_columns"])
    d.num_nodes = N
    d.num_children = _p(nc, C.c_uint32)
    d.first_child = _p(fc, C.c_uint32)
    d.leaf_column = _p(lc, C.c_uint32)
    d.vec_size = _p(vs, C.c_uint64)
    d.vec_words = ptrs
    return d, (nc, fc, lc, vs, words, ptrs)


def _tree_dict(handle):
    """Copy an mbrwt_tree (include/mbrwt.h) into a BFS tree dict and free it."""
    lib = L.lib()
    try:
        d = lib.mbrwt_tree_get_desc(handle).contents
        N = int(d.num_nodes)
        out = dict(num_rows=int(d.num_rows), num_columns=int(d.num_columns), num_nodes=N)
        for key, dt in (("num_children", np.uint32), ("first_child", np.uint32), ("leaf_column", np.uint32),
                        ("vec_size", np.uint64)):
            ptr = getattr(d, key)
            out[key] = np.ctypeslib.as_array(ptr, shape=(N,)).astype(dt).copy() if N else np.zeros(0, dtype=dt)
        words = []
        for u in range(N):
            W = (int(out["vec_size"][u]) + 63) // 64
            words.append(np.ctypeslib.as_array(d.vec_words[u], shape=(W,)).copy() if W else
                         np.zeros(0, dtype=np.uint64))
        out["words"] = words
        return out
    finally:
        lib.mbrwt_tree_free(handle)


def parse_brwt(data: bytes):
    """BRWT::load (BRWT.cpp:87-111) of a reference BRWT stream -> (tree dict,
    bytes consumed).  Host only (include/mbrwt.h mbrwt_tree_parse)."""
    buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, dtype=np.uint8)
    h = C.c_void_p()
    used = C.c_uint64(0)
    L.check(L.lib().mbrwt_tree_parse(_p(buf, C.c_uint8), len(data), C.byref(used), C.byref(h)), "mbrwt_tree_parse")
    return _tree_dict(h), int(used.value)


def serialize_tree(tree) -> bytes:
    """BRWT::serialize (BRWT.cpp:113-128) of a tree dict.  Host only."""
    lib = L.lib()
    d, keep = tree_desc(tree)
    need = C.c_uint64(0)
    st = lib.mbrwt_tree_serialize(C.byref(d), None, 0, C.byref(need))
    if st != L.MBRWT_ERR_CAPACITY:
        L.check(st, "mbrwt_tree_serialize")
    buf = np.zeros(max(1, need.value), dtype=np.uint8)
    L.check(lib.mbrwt_tree_serialize(C.byref(d), _p(buf, C.c_uint8), len(buf), C.byref(need)), "mbrwt_tree_serialize")
    del keep
    return buf[: need.value].tobytes()


@contextlib.contextmanager
def build_layout(layout):
    """Device layout of the contexts created inside the block (None: the
    library default; 'nodes', 'rows', 'both' -- include/mbrwt.h)."""
    if layout is None:
        yield
        return
    with build_option(L.MBRWT_BUILD_LAYOUT, L.LAYOUTS[layout]):
        yield


@contextlib.contextmanager
def build_option(option, value):
    """mbrwt_set_build_option for the block; the calling thread's previous
    value is restored afterwards (mbrwt_get_build_option)."""
    lib = L.lib()
    prev = C.c_int64(0)
    L.check(lib.mbrwt_get_build_option(option, C.byref(prev)), "mbrwt_get_build_option")
    L.check(lib.mbrwt_set_build_option(option, int(value)), "mbrwt_set_build_option")
    try:
        yield
    finally:
        lib.mbrwt_set_build_option(option, prev.value)


class BRWTDevice:
    """A BRWT held in HBM; every query runs the HIP traversal kernels."""

    def __init__(self, handle, keepalive=None):
        self._h = handle
        self._keep = keepalive

    # -- construction -------------------------------------------------------
    @classmethod
    def from_tree(cls, tree, device=0, relax_max_arity=0, layout=None):
        """`tree`: BFS description (keys as include/mbrwt.h mbrwt_tree_desc:
        num_rows, num_columns, num_children, first_child, leaf_column,
        vec_size, words = list of uint64 arrays).  relax_max_arity > 1 runs
        BRWTOptimizer::relax on it first (mbrwt_create_relaxed)."""
        lib = L.lib()
        d, keep = tree_desc(tree)
        h = C.c_void_p()
        with build_layout(layout):
            if relax_max_arity:
                L.check(lib.mbrwt_create_relaxed(C.byref(d), int(relax_max_arity), device, C.byref(h)),
                        "mbrwt_create_relaxed")
            else:
                L.check(lib.mbrwt_create(C.byref(d), device, C.byref(h)), "mbrwt_create")
        return cls(h)

    @classmethod
    def synthetic(cls, num_rows, num_columns, density, arity=8, seed=42, device=0, layout=None):
        lib = L.lib()
        d = L.SynthDesc(num_rows, num_columns, float(density), arity, seed)
        h = C.c_void_p()
        with build_layout(layout):
            L.check(lib.mbrwt_create_synthetic(C.byref(d), device, C.byref(h)), "mbrwt_create_synthetic")
        return cls(h)

    @classmethod
    def synthetic_shaped(cls, num_rows, shape, density, seed=42, device=0, layout=None):
        """The synthetic law over a given tree shape (mbrwt_create_synthetic_shaped):
        `shape` = dict with num_children, first_child, leaf_column (BFS), e.g.
        the export of a greedy + relaxed tree."""
        lib = L.lib()
        nc = np.ascontiguousarray(shape["num_children"], dtype=np.uint32)
        fc = np.ascontiguousarray(shape["first_child"], dtype=np.uint32)
        lc = np.ascontiguousarray(shape["leaf_column"], dtype=np.uint32)
        m = int((nc == 0).sum())
        d = L.SynthDesc(num_rows, m, float(density), 0, seed)
        sd = L.ShapeDesc(len(nc), _p(nc, C.c_uint32), _p(fc, C.c_uint32), _p(lc, C.c_uint32))
        h = C.c_void_p()
        with build_layout(layout):
            L.check(lib.mbrwt_create_synthetic_shaped(C.byref(d), C.byref(sd), device, C.byref(h)),
                    "mbrwt_create_synthetic_shaped")
        return cls(h)

    @classmethod
    def from_columns(cls, columns, num_rows, arity=2, device=0, relax_max_arity=0, layout=None,
                     partitioner="basic"):
        """BRWTBottomUpBuilder::build on the device (include/mbrwt.h
        mbrwt_create_from_columns) with the basic partitioner of `arity` or,
        partitioner='greedy', binary_grouping_greedy (MBRWT_BUILD_PARTITIONER).
        `columns`: a sequence of uint64 arrays (ceil(num_rows/64) LSB-first
        words each), or a 2-D uint64 array [num_columns, words].
        relax_max_arity > 1 then runs BRWTOptimizer::relax
        (mbrwt_create_from_columns_relaxed)."""
        lib = L.lib()
        cols = [np.ascontiguousarray(c, dtype=np.uint64) for c in columns]
        W = (num_rows + 63) // 64
        if any(len(c) < W for c in cols):
            raise ValueError("a column has fewer than ceil(num_rows/64) words")
        ptrs = (L.u64p * max(1, len(cols)))()
        for j, c in enumerate(cols):
            ptrs[j] = c.ctypes.data_as(L.u64p)
        d = L.ColumnsDesc(num_rows, len(cols), ptrs, arity)
        h = C.c_void_p()
        with build_option(L.MBRWT_BUILD_PARTITIONER, L.PARTITIONERS[partitioner]), build_layout(layout):
            if relax_max_arity:
                L.check(lib.mbrwt_create_from_columns_relaxed(C.byref(d), int(relax_max_arity), device,
                                                              C.byref(h)), "mbrwt_create_from_columns_relaxed")
            else:
                L.check(lib.mbrwt_create_from_columns(C.byref(d), device, C.byref(h)), "mbrwt_create_from_columns")
        return cls(h)

    @classmethod
    def load(cls, data: bytes, device=0, layout=None):
        """BRWT::load of a reference BRWT stream into HBM (mbrwt_load)."""
        buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, dtype=np.uint8)
        h = C.c_void_p()
        with build_layout(layout):
            L.check(L.lib().mbrwt_load(_p(buf, C.c_uint8), len(data), None, device, C.byref(h)), "mbrwt_load")
        return cls(h)

    def export(self):
        """The tree this context holds, read back from its device image
        (mbrwt_tree_export), as a BFS tree dict."""
        h = C.c_void_p()
        L.check(L.lib().mbrwt_tree_export(self._h, C.byref(h)), "mbrwt_tree_export")
        return _tree_dict(h)

    def serialize(self) -> bytes:
        """BRWT::serialize (BRWT.cpp:113-128) of this matrix."""
        return serialize_tree(self.export())

    def clone(self) -> "BRWTDevice":
        """A second query context over the same device image
        (mbrwt_ctx_clone): its own workspaces, so its queries may run
        concurrently with this one's on another stream or thread."""
        h = C.c_void_p()
        L.check(L.lib().mbrwt_ctx_clone(self._h, C.byref(h)), "mbrwt_ctx_clone")
        return BRWTDevice(h.value)

    def close(self):
        if getattr(self, "_h", None):
            L.lib().mbrwt_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- properties -----------------------------------------------------------
    def num_rows(self):
        return L.lib().mbrwt_num_rows(self._h)

    def num_columns(self):
        return L.lib().mbrwt_num_columns(self._h)

    def num_relations(self):
        return L.lib().mbrwt_num_relations(self._h)

    def num_nodes(self):
        return L.lib().mbrwt_num_nodes(self._h)

    def num_shards(self):
        """Row shards of the context (1 below 2^32 rows; include/mbrwt.h)."""
        return L.lib().mbrwt_num_shards(self._h)

    def device_bytes(self):
        return L.lib().mbrwt_device_bytes(self._h)

    def layout(self):
        """'nodes', 'rows' or 'both' (include/mbrwt.h "device layout")."""
        return L.LAYOUT_NAMES.get(L.lib().mbrwt_layout(self._h), "?")

    def rows_stats(self):
        """The row-record image (mbrwt_rows_stats) as a dict, None without one."""
        out = (C.c_uint64 * 8)()
        if L.lib().mbrwt_rows_stats(self._h, out) != L.MBRWT_OK:
            return None
        keys = ("block_bytes", "rows_per_block", "blocks_bytes", "spill_bytes", "record_bytes", "spilled_rows",
                "long_rows", "height")
        d = dict(zip(keys, [int(v) for v in out]))
        d["uniform_levels"] = (d["height"] >> 32) & 0xFF  # odometer walk when > 0
        d["nibble_codes"] = bool((d["height"] >> 40) & 1)  # masks as nibble codes (MBRWT_BUILD_ROWS_CODE)
        d["terminal_records"] = bool((d["height"] >> 41) & 1)  # terminal records (MBRWT_BUILD_ROWS_CODE = 2)
        d["variable"] = d["block_bytes"] == 0  # variable-length records (csrc/rows_var.hip)
        d["height"] &= 0xFFFFFFFF
        cl = (C.c_uint64 * 4)()
        if L.lib().mbrwt_rows_classes(self._h, cl) == L.MBRWT_OK:
            # record classes (csrc/rows_class.hip): 0 = none
            d["classes"], d["class_bits"], d["class_index_bytes"], d["class_sample_distinct"] = (int(v) for v in cl)
        return d

    # -- host-buffer queries --------------------------------------------------
    def get_rows(self, rows):
        """Batched BRWT::get_row (BRWT.cpp:26-53) -> (offsets[n+1], cols)."""
        lib = L.lib()
        rows = np.ascontiguousarray(rows, dtype=np.uint64)
        n = len(rows)
        offsets = np.zeros(n + 1, dtype=np.uint64)
        need = C.c_uint64(0)
        cap = max(16, n * 16)
        while True:
            cols = np.zeros(cap, dtype=np.uint32)
            st = lib.mbrwt_get_rows(self._h, _p(rows, C.c_uint64), n, _p(offsets, C.c_uint64),
                                    _p(cols, C.c_uint32), cap, C.byref(need))
            if st == L.MBRWT_ERR_CAPACITY:
                cap = int(need.value)
                continue
            L.check(st, "mbrwt_get_rows")
            return offsets, cols[: need.value]

    def get_row(self, row):
        off, cols = self.get_rows(np.array([row], dtype=np.uint64))
        return cols.tolist()

    def get_batch(self, rows, cols):
        """Batched BRWT::get (BRWT.cpp:9-24)."""
        rows = np.ascontiguousarray(rows, dtype=np.uint64)
        cols = np.ascontiguousarray(cols, dtype=np.uint64)
        out = np.zeros(max(1, len(rows)), dtype=np.uint8)
        L.check(L.lib().mbrwt_get_batch(self._h, _p(rows, C.c_uint64), _p(cols, C.c_uint64), len(rows),
                                        _p(out, C.c_uint8)), "mbrwt_get_batch")
        return out[: len(rows)].astype(bool)

    def get(self, row, col):
        return bool(self.get_batch([row], [col])[0])

    def get_column(self, col):
        """BRWT::get_column (BRWT.cpp:55-85): ascending rows carrying `col`."""
        need = C.c_uint64(0)
        st = L.lib().mbrwt_get_column(self._h, int(col), None, 0, C.byref(need))
        if st != L.MBRWT_ERR_CAPACITY:
            L.check(st, "mbrwt_get_column")
            return np.zeros(0, dtype=np.uint64)
        out = np.zeros(max(1, need.value), dtype=np.uint64)
        L.check(L.lib().mbrwt_get_column(self._h, int(col), _p(out, C.c_uint64), len(out), C.byref(need)),
                "mbrwt_get_column")
        return out[: need.value]

    def get_column_device(self, col, rows_t, stream=None):
        """Device variant: rows_t = 64-bit cuda tensor of capacity >= the column's
        size.  Returns the number of rows written; raises on capacity."""
        need = C.c_uint64(0)
        st = L.lib().mbrwt_get_column_device(self._h, int(col), rows_t.data_ptr(), rows_t.numel(), C.byref(need),
                                             stream if stream is not None else None)
        if st == L.MBRWT_ERR_CAPACITY:
            e = L.MBRWTError(st, "mbrwt_get_column_device")
            e.needed = int(need.value)
            raise e
        L.check(st, "mbrwt_get_column_device")
        return int(need.value)

    # -- device-buffer queries (torch tensors as plumbing) ---------------------
    def get_rows_device(self, rows_t, offsets_t, cols_t, stream=None):
        """rows_t: uint64/int64 cuda tensor [n]; offsets_t: [n+1] 64-bit; cols_t:
        int32 [cap].  Returns the number of labels; raises on capacity."""
        need = C.c_uint64(0)
        st = L.lib().mbrwt_get_rows_device(self._h, rows_t.data_ptr(), rows_t.numel(), offsets_t.data_ptr(),
                                           cols_t.data_ptr(), cols_t.numel(), C.byref(need),
                                           stream if stream is not None else None)
        if st == L.MBRWT_ERR_CAPACITY:
            e = L.MBRWTError(st, "mbrwt_get_rows_device")
            e.needed = int(need.value)
            raise e
        L.check(st, "mbrwt_get_rows_device")
        return int(need.value)

    def get_rows_device_async(self, rows_t, offsets_t, cols_t, status_t, stream=None):
        """mbrwt_get_rows_device_async: enqueue only; status_t (device, 3 x
        int64) receives {labels needed, status, sticky status bits}."""
        L.check(L.lib().mbrwt_get_rows_device_async(self._h, rows_t.data_ptr(), rows_t.numel(), offsets_t.data_ptr(),
                                                    cols_t.data_ptr(), cols_t.numel(), status_t.data_ptr(), stream),
                "mbrwt_get_rows_device_async")

    def get_batch_device(self, rows_t, cols_t, out_t, stream=None):
        L.check(L.lib().mbrwt_get_batch_device(self._h, rows_t.data_ptr(), cols_t.data_ptr(), rows_t.numel(),
                                               out_t.data_ptr(), stream), "mbrwt_get_batch_device")

    def count_labels_device(self, rows_t, counts_t, stream=None):
        L.check(L.lib().mbrwt_count_labels_device(self._h, rows_t.data_ptr(), rows_t.numel(), counts_t.data_ptr(),
                                                  stream), "mbrwt_count_labels_device")

    def get_labels_batch_device(self, rows_t, read_off_t, presence_ratio, lab_off_t, labels_t, stream=None):
        """get_labels(indices, presence_ratio) for many reads (include/mbrwt.h
        mbrwt_get_labels_batch_device); torch device tensors; returns the
        label count (raises MBRWTError with .needed on MBRWT_ERR_CAPACITY)."""
        need = C.c_uint64(0)
        st = L.lib().mbrwt_get_labels_batch_device(
            self._h, rows_t.data_ptr(), rows_t.numel(), read_off_t.data_ptr(), read_off_t.numel() - 1,
            float(presence_ratio), lab_off_t.data_ptr(), labels_t.data_ptr() if labels_t is not None else None,
            labels_t.numel() if labels_t is not None else 0, C.byref(need), stream)
        if st == L.MBRWT_ERR_CAPACITY:
            e = L.MBRWTError(st, "mbrwt_get_labels_batch_device")
            e.needed = int(need.value)
            raise e
        L.check(st, "mbrwt_get_labels_batch_device")
        return int(need.value)

    def get_labels_batch(self, rows, read_offsets, presence_ratio):
        """Host-buffer form (include/mbrwt.h mbrwt_get_labels_batch): numpy in,
        (label offsets u64 [n_reads+1], labels u32) out."""
        return _labels_batch("mbrwt_get_labels_batch", self._h, rows, read_offsets, presence_ratio)

    def get_top_labels_batch(self, rows, read_offsets, num_top=2**64 - 1):
        """MultiLabelEncoded::get_top_labels(indices, num_top) for many reads
        (include/mbrwt.h mbrwt_get_top_labels_batch): -> (label offsets u64
        [n_reads+1], labels u32, counts u64), each read by count descending,
        equal counts by label ascending."""
        return _top_labels_batch("mbrwt_get_top_labels_batch", self._h, rows, read_offsets, num_top)

    def get_top_labels_batch_device(self, rows_t, read_off_t, num_top, lab_off_t, labels_t, counts_t, stream=None):
        """Device-buffer form on torch tensors (labels int32, counts int64);
        returns the label count (raises MBRWTError with .needed on capacity)."""
        need = C.c_uint64(0)
        out = labels_t is not None and counts_t is not None
        st = L.lib().mbrwt_get_top_labels_batch_device(
            self._h, rows_t.data_ptr(), rows_t.numel(), read_off_t.data_ptr(), read_off_t.numel() - 1, int(num_top),
            lab_off_t.data_ptr(), labels_t.data_ptr() if out else None, counts_t.data_ptr() if out else None,
            min(labels_t.numel(), counts_t.numel()) if out else 0, C.byref(need), stream)
        if st == L.MBRWT_ERR_CAPACITY:
            e = L.MBRWTError(st, "mbrwt_get_top_labels_batch_device")
            e.needed = int(need.value)
            raise e
        L.check(st, "mbrwt_get_top_labels_batch_device")
        return int(need.value)

    def count_work_device(self, rows_t, stream=None):
        v = C.c_uint64(0)
        lab = C.c_uint64(0)
        L.check(L.lib().mbrwt_count_work_device(self._h, rows_t.data_ptr(), rows_t.numel(), C.byref(v),
                                                C.byref(lab), stream), "mbrwt_count_work_device")
        return int(v.value), int(lab.value)

    # -- options / measurement ------------------------------------------------
    def set_option(self, option, value):
        L.check(L.lib().mbrwt_set_option(self._h, option, int(value)), "mbrwt_set_option")

    def traverse_kernel(self) -> str:
        """Name of the traversal kernel get_rows launches (diagnostics)."""
        return (L.lib().mbrwt_traverse_kernel(self._h) or b"").decode()

    def take_timing(self):
        ms = C.c_double(0)
        k = C.c_uint64(0)
        L.check(L.lib().mbrwt_take_timing(self._h, C.byref(ms), C.byref(k)), "mbrwt_take_timing")
        return ms.value, int(k.value)


class BRWTMulti:
    """One replica per device, get_rows over all of them (include/mbrwt.h
    "multi-device"): the batch is cut into contiguous slices, one per replica,
    and reassembled into one CSR."""

    def __init__(self, handle, keepalive=None):
        self._h = handle
        self._keep = keepalive

    @classmethod
    def from_tree(cls, tree, devices=(0,), layout=None):
        lib = L.lib()
        d, keep = tree_desc(tree)
        devs = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        with build_layout(layout):
            L.check(lib.mbrwt_multi_create(C.byref(d), devs, len(devices), C.byref(h)), "mbrwt_multi_create")
        return cls(h)

    @classmethod
    def synthetic(cls, num_rows, num_columns, density, arity=8, seed=42, devices=(0,), layout=None):
        lib = L.lib()
        d = L.SynthDesc(num_rows, num_columns, float(density), arity, seed)
        devs = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        with build_layout(layout):
            L.check(lib.mbrwt_multi_create_synthetic(C.byref(d), devs, len(devices), C.byref(h)),
                    "mbrwt_multi_create_synthetic")
        return cls(h)

    def close(self):
        if getattr(self, "_h", None):
            L.lib().mbrwt_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def size(self):
        return L.lib().mbrwt_multi_size(self._h)

    def replica(self, i):
        """Replica i as a BRWTDevice view (owned by this handle)."""
        h = L.lib().mbrwt_multi_replica(self._h, i)
        if not h:
            raise IndexError(i)
        dev = BRWTDevice.__new__(BRWTDevice)
        dev._h = C.c_void_p(h)
        dev._keep = self
        dev.close = lambda: None  # the multi handle owns it
        return dev

    def get_rows(self, rows):
        lib = L.lib()
        rows = np.ascontiguousarray(rows, dtype=np.uint64)
        n = len(rows)
        offsets = np.zeros(n + 1, dtype=np.uint64)
        need = C.c_uint64(0)
        cap = max(16, n * 16)
        while True:
            cols = np.zeros(cap, dtype=np.uint32)
            st = lib.mbrwt_multi_get_rows(self._h, _p(rows, C.c_uint64), n, _p(offsets, C.c_uint64),
                                          _p(cols, C.c_uint32), cap, C.byref(need))
            if st == L.MBRWT_ERR_CAPACITY:
                cap = int(need.value)
                continue
            L.check(st, "mbrwt_multi_get_rows")
            return offsets, cols[: need.value]

    def get_rows_device(self, rows_t, offsets_t, cols_t, stream=None):
        need = C.c_uint64(0)
        st = L.lib().mbrwt_multi_get_rows_device(self._h, rows_t.data_ptr(), rows_t.numel(), offsets_t.data_ptr(),
                                                 cols_t.data_ptr(), cols_t.numel(), C.byref(need), stream)
        if st == L.MBRWT_ERR_CAPACITY:
            e = L.MBRWTError(st, "mbrwt_multi_get_rows_device")
            e.needed = int(need.value)
            raise e
        L.check(st, "mbrwt_multi_get_rows_device")
        return int(need.value)
