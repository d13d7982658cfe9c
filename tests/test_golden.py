"""Committed golden fixtures (tests/golden/, made by make_golden.py):
the oracle must keep reproducing them (CPU), and the HIP engine must match
them bit for bit through the C ABI (GPU)."""
import os

import numpy as np
import pytest

from conftest import gpu_available

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NOREPL = ["c1_norepl_small.npz", "c2_kingsford_small.npz"]
DENSE = ["greedy_relax_small.npz", "basic_relax_unbounded.npz"]


def _load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def _oracle_tree(O, name):
    f = _load(name)
    if name in NOREPL:
        return f, O.OracleTree.norepl(int(f["n"]), int(f["m"]), float(f["d"]), 42, str(f["partitioner"]),
                                      int(f["arity"]))
    if name in DENSE:
        dense = np.unpackbits(f["dense"], axis=1)[:, : int(f["m"])].astype(bool)
        return f, O.OracleTree.from_dense(dense, str(f["partitioner"]), int(f["arity"]), int(f["relax"]))
    return f, O.OracleTree.topdown(int(f["n"]), int(f["m"]), float(f["d"]), int(f["arity"]), 42)


@pytest.mark.parametrize("name", NOREPL + DENSE + ["synth_kingsford_small.npz"])
def test_oracle_reproduces_golden(oracle_mod, name):
    f, t = _oracle_tree(oracle_mod, name)
    off, cols = t.get_rows(f["rows"])
    np.testing.assert_array_equal(off, f["offsets"])
    np.testing.assert_array_equal(cols, f["cols"])
    if "hashes" in f:
        hs = [oracle_mod.synth_hash(42, k, p) for k in (0, 1, 0xFFFFFFFF) for p in (0, 1, 12345, 2**32 - 1)]
        np.testing.assert_array_equal(np.array(hs, dtype=np.uint64), f["hashes"])


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a GPU")
@pytest.mark.parametrize("name", NOREPL + DENSE + ["synth_kingsford_small.npz"])
def test_device_matches_golden(oracle_mod, name):
    from genome_graph_annotation_amd import BRWTDevice
    f, t = _oracle_tree(oracle_mod, name)
    if name.startswith("synth"):
        d = BRWTDevice.synthetic(int(f["n"]), int(f["m"]), float(f["d"]), int(f["arity"]), 42)
        assert d.num_relations() == int(f["num_relations"])
    else:
        d = BRWTDevice.from_tree(t.export())
    off, cols = d.get_rows(f["rows"])
    np.testing.assert_array_equal(off, f["offsets"])
    np.testing.assert_array_equal(cols, f["cols"])
