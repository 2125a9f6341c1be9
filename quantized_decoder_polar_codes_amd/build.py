"""In-tree build of libqpd.so (HIP, gfx950).  No JIT cache, no site-packages:
the .so lands next to this file so it travels to the GPU box with the repo."""
from __future__ import annotations

import hashlib
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


# Translation units and their own flags (compiled in parallel): the C-ABI (host
# code, the pre-pass / Monte-Carlo / probe kernels), the decode kernel
# instantiations of SC/SCL/FastSC-LUT and of FastSCL-LUT (one template,
# qpd_fast.hip), the generic engine's, the LUT generator.
UNITS = [
    ("qpd_capi.hip", []),
    ("qpd_k_fast.hip", []),
    ("qpd_k_scl.hip", []),
    ("qpd_k_scl1.hip", []),
    ("qpd_fast_fscl.hip", []),
    ("qpd_fast_fscl1.hip", []),
    ("qpd_k_generic.hip", []),
    ("qpd_lutgen.cpp", []),
]
COMMON_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function"]


def source_hash() -> str:
    """SHA-256 over every source file, the target and the compile flags: the
    build id stamped into libqpd.so (qpd_build_id) and checked when the
    library is loaded, so a shipped binary provably matches the tree."""
    h = hashlib.sha256()
    h.update(repr((ARCH, COMMON_FLAGS, UNITS)).encode())
    for path in _sources():
        h.update(os.path.relpath(path, ROOT).encode() + b"\0")
        with open(path, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:32]


BUILD_ID_TAG = b"qpd-build-id:"


def library_build_id(path: str = LIB) -> str | None:
    """The build id embedded in a built library (read from its bytes, no dlopen)."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(BUILD_ID_TAG)
    if i < 0:
        return None
    return data[i + len(BUILD_ID_TAG): i + len(BUILD_ID_TAG) + 32].decode("ascii", "replace")


def needs_build() -> bool:
    return library_build_id() != source_hash()


def build_native(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return LIB
    bid = source_hash()
    common = [HIPCC, f"--offload-arch={ARCH}"] + COMMON_FLAGS + ["-I", os.path.join(ROOT, "include"), "-I", SRC,
                                                                 f'-DQPD_BUILD_ID="{bid}"']
    objs, procs = [], []
    odir = os.path.join(ROOT, "build", "obj")  # kept: tools/build_variant.sh links variants against them
    os.makedirs(odir, exist_ok=True)
    for src, extra in UNITS:  # the units compile in parallel
        obj = os.path.join(odir, os.path.splitext(src)[0] + ".o")
        cmd = common + extra + ["-c", os.path.join(SRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        objs.append(obj)
        procs.append((cmd, subprocess.Popen(cmd)))
    for cmd, p in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC"] + objs + ["-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    with open(os.path.join(odir, "BUILD_ID"), "w") as f:  # tools/build_variant.sh links against these objects
        f.write(bid + "\n")
    return LIB


if __name__ == "__main__":
    print(build_native(force=True, verbose=True))
