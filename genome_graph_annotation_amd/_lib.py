"""ctypes binding of libmbrwt.so (include/mbrwt.h).

The binding is exactly what a reference-side maintainer would write (see
INTEGRATION.md).  There is no fallback: if the HIP library is missing the
import fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MBRWT_LIB: another build of the same library (same-box A/B of kernel changes, tools/ab.sh)
LIB_PATH = os.environ.get("MBRWT_LIB") or os.path.join(_HERE, "libmbrwt.so")

MBRWT_OK = 0
MBRWT_ERR_INVALID = 1
MBRWT_ERR_RANGE = 2
MBRWT_ERR_CAPACITY = 3
MBRWT_ERR_UNSUPPORTED = 4
MBRWT_ERR_DEVICE = 5
MBRWT_ERR_NOMEM = 6

MBRWT_OPT_TIMING = 1
MBRWT_OPT_SLOT_LABELS = 2
MBRWT_OPT_KERNEL = 4
MBRWT_OPT_ROWS_WALK = 8
MBRWT_OPT_TEST_FAIL_CHUNK = 32  # test hook (host-buffer path)
MBRWT_OPT_COMPACT_CUS = 64  # row records: compaction on a CU-masked stream (measurement)

MBRWT_BUILD_LAYOUT = 1
MBRWT_BUILD_PARTITIONER = 2
MBRWT_BUILD_ROWS_FOOTPRINT = 3
MBRWT_BUILD_ROWS_VAR = 4
MBRWT_BUILD_VAR_LANES = 5
MBRWT_BUILD_ROWS_BLOCK = 6
MBRWT_BUILD_ROWS_RANGE = 7
MBRWT_BUILD_NODE_KINDS = 8
MBRWT_BUILD_SHARD_ROWS = 9
MBRWT_BUILD_ROWS_WGS_PER_CU = 10
MBRWT_BUILD_ROWS_CLASSES = 11
MBRWT_BUILD_ROWS_CODE = 12
MBRWT_KIND_FOLD_ROOT = 1
MBRWT_KIND_PACK = 2
MBRWT_KIND_PACK2 = 4
MBRWT_KIND_PACKT = 8
MBRWT_KIND_ALL = 15
MBRWT_ROWS_FAST = 0
MBRWT_ROWS_COMPACT = 1
MBRWT_PARTITIONER_BASIC = 0
MBRWT_PARTITIONER_GREEDY = 1
PARTITIONERS = {"basic": MBRWT_PARTITIONER_BASIC, "greedy": MBRWT_PARTITIONER_GREEDY}
MBRWT_LAYOUT_AUTO = 0
MBRWT_LAYOUT_NODES = 1
MBRWT_LAYOUT_ROWS = 2
MBRWT_LAYOUT_BOTH = 3
LAYOUTS = {"auto": MBRWT_LAYOUT_AUTO, "nodes": MBRWT_LAYOUT_NODES, "rows": MBRWT_LAYOUT_ROWS,
           "both": MBRWT_LAYOUT_BOTH}
LAYOUT_NAMES = {1: "nodes", 2: "rows", 3: "both"}

u64p = C.POINTER(C.c_uint64)
u32p = C.POINTER(C.c_uint32)
u8p = C.POINTER(C.c_uint8)


class TreeDesc(C.Structure):
    _fields_ = [
        ("num_rows", C.c_uint64),
        ("num_columns", C.c_uint64),
        ("num_nodes", C.c_uint32),
        ("num_children", u32p),
        ("first_child", u32p),
        ("leaf_column", u32p),
        ("vec_size", u64p),
        ("vec_words", C.POINTER(u64p)),
    ]


class SynthDesc(C.Structure):
    _fields_ = [
        ("num_rows", C.c_uint64),
        ("num_columns", C.c_uint64),
        ("density", C.c_double),
        ("arity", C.c_uint32),
        ("seed", C.c_uint64),
    ]


class ShapeDesc(C.Structure):
    _fields_ = [
        ("num_nodes", C.c_uint32),
        ("num_children", u32p),
        ("first_child", u32p),
        ("leaf_column", u32p),
    ]


class ColumnsDesc(C.Structure):
    _fields_ = [
        ("num_rows", C.c_uint64),
        ("num_columns", C.c_uint64),
        ("columns", C.POINTER(u64p)),
        ("arity", C.c_uint32),
    ]


class BinRelDesc(C.Structure):  # include/mbrwt_wt.h
    _fields_ = [
        ("num_rows", C.c_uint64),
        ("num_columns", C.c_uint64),
        ("offsets", u64p),
        ("cols", u32p),
    ]


class BinRelSynthDesc(C.Structure):
    _fields_ = [
        ("num_rows", C.c_uint64),
        ("num_columns", C.c_uint64),
        ("density", C.c_double),
        ("seed", C.c_uint64),
    ]


# every symbol include/mbrwt.h and include/mbrwt_wt.h declare, with its signature
SIGNATURES = {
    "mbrwt_create": (C.c_int, [C.POINTER(TreeDesc), C.c_int, C.POINTER(C.c_void_p)]),
    "mbrwt_create_synthetic": (C.c_int, [C.POINTER(SynthDesc), C.c_int, C.POINTER(C.c_void_p)]),
    "mbrwt_create_synthetic_shaped": (C.c_int, [C.POINTER(SynthDesc), C.POINTER(ShapeDesc), C.c_int,
                                                C.POINTER(C.c_void_p)]),
    "mbrwt_create_from_columns": (C.c_int, [C.POINTER(ColumnsDesc), C.c_int, C.POINTER(C.c_void_p)]),
    "mbrwt_create_from_columns_relaxed": (C.c_int, [C.POINTER(ColumnsDesc), C.c_uint64, C.c_int,
                                                    C.POINTER(C.c_void_p)]),
    "mbrwt_create_relaxed": (C.c_int, [C.POINTER(TreeDesc), C.c_uint64, C.c_int, C.POINTER(C.c_void_p)]),
    "mbrwt_get_labels_batch": (C.c_int, [C.c_void_p, u64p, C.c_uint64, u64p, C.c_uint64, C.c_double, u64p, u32p,
                                         C.c_uint64, u64p]),
    "mbrwt_get_top_labels_batch": (C.c_int, [C.c_void_p, u64p, C.c_uint64, u64p, C.c_uint64, C.c_uint64, u64p,
                                             u32p, u64p, C.c_uint64, u64p]),
    "mbrwt_get_top_labels_batch_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                                    C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                                    u64p, C.c_void_p]),
    "mbrwt_get_labels_batch_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                                C.c_double, C.c_void_p, C.c_void_p, C.c_uint64, u64p, C.c_void_p]),
    "mbrwt_pack_ids_device": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p]),
    "mbrwt_unpack_ids_device": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p]),
    "mbrwt_unpack_segments_device": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint64, u64p, C.c_uint32, C.c_void_p,
                                               C.c_void_p]),
    "mbrwt_wire_labels_offset": (C.c_uint64, [C.c_uint64, C.c_uint32]),
    "mbrwt_pack_csr_device": (C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_uint32,
                                        C.c_uint32, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p]),
    "mbrwt_unpack_labels_device": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32,
                                             C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]),
    "mbrwt_unpack_offsets_device": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint64, u64p, C.c_uint32, C.c_void_p,
                                              C.c_void_p, C.POINTER(C.c_uint64), C.c_void_p]),
    "mbrwt_destroy": (None, [C.c_void_p]),
    "mbrwt_ctx_clone": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p)]),
    "mbrwt_set_build_option": (C.c_int, [C.c_int, C.c_int64]),
    "mbrwt_get_build_option": (C.c_int, [C.c_int, C.POINTER(C.c_int64)]),
    "mbrwt_multi_create": (C.c_int, [C.POINTER(TreeDesc), C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_void_p)]),
    "mbrwt_multi_create_synthetic": (C.c_int, [C.POINTER(SynthDesc), C.POINTER(C.c_int), C.c_int,
                                               C.POINTER(C.c_void_p)]),
    "mbrwt_multi_load": (C.c_int, [u8p, C.c_uint64, u64p, C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_void_p)]),
    "mbrwt_multi_destroy": (None, [C.c_void_p]),
    "mbrwt_multi_size": (C.c_int, [C.c_void_p]),
    "mbrwt_multi_replica": (C.c_void_p, [C.c_void_p, C.c_int]),
    "mbrwt_multi_get_rows": (C.c_int, [C.c_void_p, u64p, C.c_uint64, u64p, u32p, C.c_uint64, u64p]),
    "mbrwt_multi_get_rows_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                              C.c_uint64, u64p, C.c_void_p]),
    "mbrwt_layout": (C.c_int, [C.c_void_p]),
    "mbrwt_rows_stats": (C.c_int, [C.c_void_p, u64p]),
    "mbrwt_rows_classes": (C.c_int, [C.c_void_p, u64p]),
    "mbrwt_tree_parse": (C.c_int, [u8p, C.c_uint64, u64p, C.POINTER(C.c_void_p)]),
    "mbrwt_tree_serialize": (C.c_int, [C.POINTER(TreeDesc), u8p, C.c_uint64, u64p]),
    "mbrwt_tree_export": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p)]),
    "mbrwt_tree_get_desc": (C.POINTER(TreeDesc), [C.c_void_p]),
    "mbrwt_tree_free": (None, [C.c_void_p]),
    "mbrwt_load": (C.c_int, [u8p, C.c_uint64, u64p, C.c_int, C.POINTER(C.c_void_p)]),
    "mbrwt_num_rows": (C.c_uint64, [C.c_void_p]),
    "mbrwt_num_columns": (C.c_uint64, [C.c_void_p]),
    "mbrwt_num_relations": (C.c_uint64, [C.c_void_p]),
    "mbrwt_num_nodes": (C.c_uint64, [C.c_void_p]),
    "mbrwt_device_bytes": (C.c_uint64, [C.c_void_p]),
    "mbrwt_device": (C.c_int, [C.c_void_p]),
    "mbrwt_num_shards": (C.c_uint64, [C.c_void_p]),
    "mbrwt_get_rows": (C.c_int, [C.c_void_p, u64p, C.c_uint64, u64p, u32p, C.c_uint64, u64p]),
    "mbrwt_get_rows_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint64,
                                        u64p, C.c_void_p]),
    "mbrwt_get_rows_device_async": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                              C.c_uint64, C.c_void_p, C.c_void_p]),
    "mbrwt_get_column": (C.c_int, [C.c_void_p, C.c_uint64, u64p, C.c_uint64, u64p]),
    "mbrwt_get_column_device": (C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, u64p, C.c_void_p]),
    "mbrwt_get_batch": (C.c_int, [C.c_void_p, u64p, u64p, C.c_uint64, u8p]),
    "mbrwt_get_batch_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]),
    "mbrwt_count_labels_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]),
    "mbrwt_count_work_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, u64p, u64p, C.c_void_p]),
    "mbrwt_set_option": (C.c_int, [C.c_void_p, C.c_int, C.c_int64]),
    "mbrwt_take_timing": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), u64p]),
    "mbrwt_strerror": (C.c_char_p, [C.c_int]),
    "mbrwt_last_error_message": (C.c_char_p, []),
    "mbrwt_traverse_kernel": (C.c_char_p, [C.c_void_p]),
    # include/mbrwt_wt.h (BinRel-WT)
    "mbrwt_wt_create": (C.c_int, [C.POINTER(BinRelDesc), C.c_int, C.POINTER(C.c_void_p)]),
    "mbrwt_wt_create_synthetic": (C.c_int, [C.POINTER(BinRelSynthDesc), C.c_int, C.POINTER(C.c_void_p)]),
    "mbrwt_wt_parse": (C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_void_p)]),
    "mbrwt_binrel_get_desc": (C.POINTER(BinRelDesc), [C.c_void_p]),
    "mbrwt_binrel_free": (None, [C.c_void_p]),
    "mbrwt_wt_serialize_desc": (C.c_int, [C.POINTER(BinRelDesc), C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]),
    "mbrwt_wt_load": (C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64), C.c_int, C.POINTER(C.c_void_p)]),
    "mbrwt_wt_serialize": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]),
    "mbrwt_wt_destroy": (None, [C.c_void_p]),
    "mbrwt_wt_num_rows": (C.c_uint64, [C.c_void_p]),
    "mbrwt_wt_num_columns": (C.c_uint64, [C.c_void_p]),
    "mbrwt_wt_num_relations": (C.c_uint64, [C.c_void_p]),
    "mbrwt_wt_device_bytes": (C.c_uint64, [C.c_void_p]),
    "mbrwt_wt_get_rows": (C.c_int, [C.c_void_p, u64p, C.c_uint64, u64p, u32p, C.c_uint64, u64p]),
    "mbrwt_wt_get_rows_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint64,
                                           u64p, C.c_void_p]),
    "mbrwt_wt_get_labels_batch": (C.c_int, [C.c_void_p, u64p, C.c_uint64, u64p, C.c_uint64, C.c_double, u64p,
                                            u32p, C.c_uint64, u64p]),
    "mbrwt_wt_get_labels_batch_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                                   C.c_double, C.c_void_p, C.c_void_p, C.c_uint64, u64p,
                                                   C.c_void_p]),
    "mbrwt_wt_get_top_labels_batch": (C.c_int, [C.c_void_p, u64p, C.c_uint64, u64p, C.c_uint64, C.c_uint64, u64p,
                                                u32p, u64p, C.c_uint64, u64p]),
    "mbrwt_wt_get_top_labels_batch_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                                       C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p,
                                                       C.c_void_p, C.c_uint64, u64p, C.c_void_p]),
    "mbrwt_wt_get_batch": (C.c_int, [C.c_void_p, u64p, u64p, C.c_uint64, u8p]),
    "mbrwt_wt_get_batch_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                            C.c_void_p]),
    "mbrwt_wt_get_column": (C.c_int, [C.c_void_p, C.c_uint64, u64p, C.c_uint64, u64p]),
    "mbrwt_wt_get_column_device": (C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, u64p, C.c_void_p]),
    "mbrwt_wt_set_option": (C.c_int, [C.c_void_p, C.c_int, C.c_int64]),
    "mbrwt_wt_take_timing": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), u64p]),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(there is no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        older = bool(os.environ.get("MBRWT_LIB"))  # an A/B build of an earlier commit may lack newer entry points
        for name, (res, args) in SIGNATURES.items():
            if older and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


class MBRWTError(RuntimeError):
    def __init__(self, status, where=""):
        L = lib()
        msg = L.mbrwt_strerror(status).decode()
        detail = (L.mbrwt_last_error_message() or b"").decode()
        super().__init__(f"{where}: {msg} ({detail})" if where else f"{msg} ({detail})")
        self.status = status


def check(status, where=""):
    if status != MBRWT_OK:
        raise MBRWTError(status, where)
