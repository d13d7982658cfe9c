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
