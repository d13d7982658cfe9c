import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: large-size case")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle as O
    O.build()
    return O


@pytest.fixture
def nodes_layout():
    """Pin the calling thread's build layout to the per-node images: the
    tests of the node kernels, image kinds and row shards.  The library
    default (AUTO) builds row records wherever they apply."""
    from genome_graph_annotation_amd.brwt import build_layout
    with build_layout("nodes"):
        yield


# ---- build options (include/mbrwt.h MBRWT_BUILD_*): scoped per test --------
# The r04 environment switches of the library are build options since r05;
# tests name them by their old switch names, translated here.
def _build_option_of(name, value):
    from genome_graph_annotation_amd import _lib as L
    import ctypes as C
    kinds = {"MBRWT_PACK": L.MBRWT_KIND_PACK, "MBRWT_PACK2": L.MBRWT_KIND_PACK2, "MBRWT_PACKT": L.MBRWT_KIND_PACKT,
             "MBRWT_FOLD_ROOT": L.MBRWT_KIND_FOLD_ROOT}
    value = str(value)
    if name in kinds:
        cur = C.c_int64(0)
        L.check(L.lib().mbrwt_get_build_option(L.MBRWT_BUILD_NODE_KINDS, C.byref(cur)), "mbrwt_get_build_option")
        bit = kinds[name]
        return L.MBRWT_BUILD_NODE_KINDS, (cur.value | bit) if value != "0" else (cur.value & ~bit)
    if name == "MBRWT_ROWS_BS":
        b, s = (int(x) for x in value.split(","))
        return L.MBRWT_BUILD_ROWS_BLOCK, b << 8 | s
    if name == "MBRWT_LAYOUT":
        return L.MBRWT_BUILD_LAYOUT, L.LAYOUTS[value]
    table = {"MBRWT_ROWS_VAR": L.MBRWT_BUILD_ROWS_VAR, "MBRWT_VAR_G": L.MBRWT_BUILD_VAR_LANES,
             "MBRWT_ROWS_RANGE": L.MBRWT_BUILD_ROWS_RANGE, "MBRWT_SHARD_ROWS": L.MBRWT_BUILD_SHARD_ROWS,
             "MBRWT_ROWS_WGS_PER_CU": L.MBRWT_BUILD_ROWS_WGS_PER_CU, "MBRWT_ROWS_CODE": L.MBRWT_BUILD_ROWS_CODE}
    return table[name], int(value)


def with_build(name, value, fn):
    """fn() with the build option `name` (an r04 switch name) set to value."""
    from genome_graph_annotation_amd.brwt import build_option
    opt, v = _build_option_of(name, value)
    with build_option(opt, v):
        return fn()


@pytest.fixture
def build_env():
    """build_env(name, value): set a build option for the rest of the test
    (restored afterwards), in place of monkeypatch.setenv on the r04 switch."""
    import contextlib
    from genome_graph_annotation_amd.brwt import build_option
    with contextlib.ExitStack() as stack:
        def set_(name, value):
            opt, v = _build_option_of(name, value)
            stack.enter_context(build_option(opt, v))
        yield set_


def kernel_variants(dev, variants):
    """The MBRWT_OPT_KERNEL values of `variants` this library accepts on dev:
    the release build dispatches 0 and 1 only (the measured A/B variants are
    an A/B build, -DMBRWT_AB_VARIANTS); restores variant 0."""
    from genome_graph_annotation_amd import _lib as L
    ok = []
    for v in variants:
        if L.lib().mbrwt_set_option(dev._h, L.MBRWT_OPT_KERNEL, int(v)) == L.MBRWT_OK:
            ok.append(v)
    L.lib().mbrwt_set_option(dev._h, L.MBRWT_OPT_KERNEL, 0)
    return ok
