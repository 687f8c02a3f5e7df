"""Builds the in-tree HIP extension ``sds_amd/lib/libsdsj.so`` for gfx950 with hipcc.

Plain ``hipcc -shared -fPIC`` (no torch extension machinery): the library exposes the C-ABI of
``include/sdsj.h`` and is loaded with ctypes after ``import torch`` so the process keeps a single
HIP runtime (torch's ``libamdhip64.so.7``, same SONAME as /opt/rocm's).
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIB_DIR, "libsdsj.so")
ARCH = os.environ.get("SDSJ_OFFLOAD_ARCH", "gfx950")


def sources() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def deps() -> list[str]:
    return sources() + sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(REPO, "include", "sdsj.h")]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the MI355X extension cannot be built")


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(p) <= t for p in deps())


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and up_to_date():
        return LIB
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = LIB + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-ffp-contract=off", "-Wl,-z,defs", "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
           "-I", os.path.join(REPO, "include"), "-o", tmp] + os.environ.get("SDSJ_CFLAGS", "").split() + sources()
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True, verbose=True))
