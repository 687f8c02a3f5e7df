"""The C-ABI library loads and exports every symbol include/sdsj.h declares (no GPU needed)."""
import os
import re
import subprocess

import pytest

from oracle import oracle as O
from tests import goldens as G

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    text = open(os.path.join(REPO, "include", "sdsj.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(sdsj_\w+)\(", text, re.M)))


def test_header_declares_expected_entry_points():
    syms = header_symbols()
    for s in ("sdsj_probe", "sdsj_engine_create", "sdsj_decode_resize_batch", "sdsj_decode_resize_batch_device"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from sds_amd import _lib
    lib = _lib.load()
    for s in header_symbols():
        assert hasattr(lib, s), s
    assert sorted(_lib.EXPORTS) == header_symbols()
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\b(sdsj_\w+)\b", out))
    assert set(header_symbols()) <= exported
    assert lib.sdsj_abi_version() == _lib.SDSJ_ABI_VERSION


def test_library_is_gfx950_code_object():
    from sds_amd import _lib
    _lib.load()
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


G1 = list(G.g1())


@pytest.mark.parametrize("case,jpg,arrs", G1, ids=[c["name"] for c, _, _ in G1])
def test_host_probe_matches_oracle(case, jpg, arrs):
    from sds_amd import _lib
    st, info = _lib.probe(jpg)
    ost, oinfo = O.probe(jpg)
    if case["name"].startswith("truncated"):
        return  # the header is intact; truncation is detected by the decode
    assert st == ost
    if st == 0:
        assert (info.width, info.height, info.ncomp) == (oinfo.width, oinfo.height, oinfo.ncomp)
        assert list(info.h_samp)[: info.ncomp] == list(oinfo.h)[: info.ncomp]
        assert info.entropy_offset == oinfo.entropy_offset
        assert info.supported == 1
        assert [info.width, info.height] == case["size"]


def test_probe_rejects_garbage():
    """Input that is not a JPEG stream (no SOI) is another format PIL would open (sds/structs.py:42
    IMAGE_EXT): unsupported by this path.  A JPEG cut inside its first marker is corrupt."""
    from sds_amd import _lib
    assert _lib.probe(b"")[0] == _lib.UNSUPPORTED
    assert _lib.probe(b"\x89PNG\r\n\x1a\n" + b"\0" * 64)[0] == _lib.UNSUPPORTED
    assert _lib.probe(b"\xff\xd8\xff")[0] == _lib.CORRUPT
