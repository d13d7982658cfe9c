"""The C++ host mirror (csrc/brwt_device.hpp, csrc/annotate_static.hpp,
csrc/binrel_wt_device.hpp) runs the reference's own test cases (test_BRWT.cpp,
test_BRWT_optimizer.cpp, test_annotation_BRWT.cpp, test_bin_rel_wt_sdsl.cpp) -- on the CPU oracle here, on the GPU engine
through the C ABI under -m gpu."""
import os
import subprocess

import pytest

from conftest import gpu_available

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")


@pytest.fixture(scope="module")
def binaries(oracle_mod):
    subprocess.run(["make", "-s", "-C", CPP], check=True)
    return os.path.join(CPP, "_build")


@pytest.mark.parametrize("prog", ["test_annotation", "test_brwt", "test_binrel_wt"])
def test_mirror_on_oracle(binaries, prog):
    r = subprocess.run([os.path.join(binaries, prog), "oracle"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed checks" in r.stdout


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a GPU")
@pytest.mark.parametrize("prog", ["test_annotation", "test_brwt", "test_binrel_wt"])
def test_mirror_on_device(binaries, prog):
    r = subprocess.run([os.path.join(binaries, prog), "device"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed checks" in r.stdout
