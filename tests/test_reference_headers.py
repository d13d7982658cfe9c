"""The C++ mirror against the reference's OWN interface header.

common/annotate.hpp (MultiLabelAnnotation / MultiLabelEncoded /
LabelEncoder) includes only the standard library, so it compiles here as it
lies under /root/reference: tests/cpp/reference_headers_check.cpp is compiled
(-fsyntax-only, templates instantiated) with MBRWT_WITH_REFERENCE_ANNOTATE
against it, proving that StaticBinRelAnnotator<BRWTDevice> is a concrete
annotate::MultiLabelEncoded.  (common/binary_matrix.hpp includes sdsl-lite,
which this image lacks, so BinaryMatrix stays restated)
Skipped where /root/reference does not exist (the GPU box).  CPU only.
"""
import os
import subprocess

import pytest

REF = "/root/reference/common"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "annotate.hpp")), reason="reference tree not present")
def test_static_annotator_is_a_reference_multilabelencoded():
    src = os.path.join(ROOT, "tests", "cpp", "reference_headers_check.cpp")
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-DMBRWT_WITH_REFERENCE_ANNOTATE", f"-I{REF}", src],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]


def test_static_annotator_restated_interface_compiles():
    """The same check against the mirror's restatement (no reference headers)."""
    src = os.path.join(ROOT, "tests", "cpp", "reference_headers_check.cpp")
    code = open(src).read().replace("annotate::", "mbrwt_host::")
    tmp = os.path.join("/tmp", "mbrwt_restated_check.cpp")
    with open(tmp, "w") as f:
        f.write(code.replace('#include "../../genome_graph_annotation_amd/csrc/annotate_static.hpp"',
                             f'#include "{ROOT}/genome_graph_annotation_amd/csrc/annotate_static.hpp"'))
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", tmp], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
