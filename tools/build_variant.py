"""Builds an experiment variant of the HIP library with extra defines (kernel A/B runs on the box).

    python tools/build_variant.py NAME -DFLAG=1 ...   ->  sds_amd/lib/exp/libsdsj_NAME.so

Run it here (hipcc cross-compiles gfx950); the .so travels with the gpurun snapshot and is selected
with SDSJ_LIBRARY=sds_amd/lib/exp/libsdsj_NAME.so.  The product library is untouched.
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from sds_amd import build as B  # noqa: E402


def main() -> None:
    name, flags = sys.argv[1], sys.argv[2:]
    out_dir = os.path.join(REPO, "sds_amd", "lib", "exp")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, f"libsdsj_{name}.so")
    cmd = [B.hipcc(), f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
           "-Wl,-z,defs", "-w", "-I", os.path.join(REPO, "include"), "-o", out] + flags + B.sources()
    subprocess.run(cmd, check=True)
    print(out)


if __name__ == "__main__":
    main()
