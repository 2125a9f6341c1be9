"""In-tree build of libqpd.so (HIP, gfx950).  No JIT cache, no site-packages:
the .so lands next to this file so it travels to the GPU box with the repo."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libqpd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("QPD_OFFLOAD_ARCH", "gfx950")


def _sources():
    return [os.path.join(SRC, f) for f in sorted(os.listdir(SRC))] + [os.path.join(ROOT, "include", "qpd.h")]


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(s) > t for s in _sources())


def build_native(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return LIB
    cmd = [
        HIPCC,
        f"--offload-arch={ARCH}",
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-shared",
        "-Wall",
        "-Wno-unused-function",
        "-I",
        os.path.join(ROOT, "include"),
        "-I",
        SRC,
        os.path.join(SRC, "qpd_capi.hip"),
        os.path.join(SRC, "qpd_lutgen.cpp"),
        "-o",
        LIB + ".tmp",
    ]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build_native(force=True, verbose=True))
