"""The product package never imports or links the oracle (it is test infrastructure only)."""
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_product_sources_do_not_reference_the_oracle():
    for root, _, files in os.walk(os.path.join(REPO, "sds_amd")):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                text = open(os.path.join(root, f)).read()
                assert not re.search(r"\boracle\b", text), os.path.join(root, f)


def test_library_does_not_link_the_oracle():
    import subprocess
    from sds_amd import _lib
    out = subprocess.run(["readelf", "-d", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out
