"""ctypes wrapper around the CPU restatement (oracle/qpd_oracle.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
``cpu_baseline`` leg of bench.py as the checker.  The product package never
imports this module.  Also exposes the reference decoders compiled from their
own sources (oracle/_ref, built by oracle/build_ref.sh) when that build exists.
"""
from __future__ import annotations

import ctypes
import glob
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libqpd_oracle.so")
REF_DIR = os.path.join(HERE, "_ref")

KIND = {"SC-LUT": 1, "SCL-LUT": 2, "FastSC-LUT": 3, "FastSCL-LUT": 4}

_lib = None


def build() -> None:
    """Compile the CPU restatement (and the reference, when /root/reference exists)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    subprocess.run([os.path.join(HERE, "build_ref.sh")], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        i32, i64 = ctypes.c_int32, ctypes.c_int64
        L.orc_decode_lut.argtypes = [i32, i32, i32, i32, i32, P, P, P, P, i32, P, P, i32, P, i32, P, i64, P]
        L.orc_decode_lut.restype = ctypes.c_int
        L.orc_decode_lut_ca.argtypes = [i32, i32, i32, i32, i32, i32, P, P, P, P, i32, P, P, i32, P, i32, i32, P,
                                        i32, P, i64, P]
        L.orc_decode_lut_ca.restype = ctypes.c_int
        L.orc_decode_sc_float.argtypes = [i32, i32, P, P, i64, P]
        L.orc_decode_sc_float.restype = ctypes.c_int
        L.orc_decode_float.argtypes = [i32, i32, i32, i32, P, P, i32, P, P, P, P, P, P, P, P, i32, i32, P, i32, P,
                                       i64, P]
        L.orc_decode_float.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def decode_lut(kind: str, packed, K: int, L: int, frozen, symbols, node_type=None) -> np.ndarray:
    """Decode int32 symbols [B, N] with the restated reference decoder ``kind``."""
    N = packed.N
    sym = np.ascontiguousarray(np.asarray(symbols, dtype=np.int32).reshape(-1, N))
    B = sym.shape[0]
    out = np.zeros((B, K), dtype=np.uint8)
    frozen = np.ascontiguousarray(np.asarray(frozen, dtype=np.int32))
    nt = None if node_type is None else np.ascontiguousarray(np.asarray(node_type).astype(np.int32))
    keep = (packed.lut_f, packed.f_base, packed.lut_g, packed.g_base, packed.vcl)
    rc = lib().orc_decode_lut(KIND[kind], N, K, L, packed.v, _ptr(frozen), _ptr(nt),
                              _ptr(packed.lut_f), _ptr(packed.f_base), packed.f_step,
                              _ptr(packed.lut_g), _ptr(packed.g_base), packed.g_step,
                              _ptr(packed.vcl), packed.vcl_rows, _ptr(sym), B, _ptr(out))
    del keep
    if rc != 0:
        raise RuntimeError(f"oracle decode failed rc={rc}")
    return out


# The CRC the reference CA decoders check (CASCLLUTDecoder.h:33-34,
# CAFastSCLLUTDecoder.h:29-30): CRC-24, whatever crc_n/crc_p the constructor got.
CRC24_LOC = (24, 23, 21, 20, 17, 15, 13, 12, 8, 4, 2, 1, 0)


def decode_lut_ca(kind: str, packed, K: int, A: int, L: int, frozen, symbols, node_type=None, crc_n: int = 24,
                  crc_loc=CRC24_LOC) -> np.ndarray:
    """CA-SCL-LUT / CA-FastSCL-LUT (kind "CA-SCL-LUT" / "CA-FastSCL-LUT"): uint8 [B, A]."""
    N = packed.N
    sym = np.ascontiguousarray(np.asarray(symbols, dtype=np.int32).reshape(-1, N))
    B = sym.shape[0]
    out = np.zeros((B, A), dtype=np.uint8)
    frozen = np.ascontiguousarray(np.asarray(frozen, dtype=np.int32))
    nt = None if node_type is None else np.ascontiguousarray(np.asarray(node_type).astype(np.int32))
    loc = np.ascontiguousarray(np.asarray(crc_loc, dtype=np.int32))
    base = {"CA-SCL-LUT": 2, "CA-FastSCL-LUT": 4}[kind]
    keep = (packed.lut_f, packed.f_base, packed.lut_g, packed.g_base, packed.vcl, loc)
    rc = lib().orc_decode_lut_ca(base, N, K, A, L, packed.v, _ptr(frozen), _ptr(nt),
                                 _ptr(packed.lut_f), _ptr(packed.f_base), packed.f_step,
                                 _ptr(packed.lut_g), _ptr(packed.g_base), packed.g_step,
                                 _ptr(packed.vcl), packed.vcl_rows, crc_n, _ptr(loc), len(loc), _ptr(sym), B, _ptr(out))
    del keep
    if rc != 0:
        raise RuntimeError(f"oracle decode failed rc={rc}")
    return out


def crc_encode(info, crc_n: int = 24, crc_loc=CRC24_LOC) -> np.ndarray:
    """CRC::encoding (utils.cpp:77-92) on rows of `info` (uint8 [B, A]) -> check bits [B, crc_n]."""
    info = np.atleast_2d(np.asarray(info, dtype=np.uint8))
    p = np.zeros(crc_n + 1, dtype=np.uint8)
    p[list(crc_loc)] = 1
    B, A = info.shape
    u = np.zeros((B, A + crc_n), dtype=np.uint8)
    u[:, :A] = info
    for i in range(A):
        rows = u[:, i] == 1
        u[rows, i:i + crc_n + 1] ^= p
    return u[:, A:]


def decode_sc_float(N: int, K: int, frozen, llr) -> np.ndarray:
    x = np.ascontiguousarray(np.asarray(llr, dtype=np.float64).reshape(-1, N))
    out = np.zeros((x.shape[0], K), dtype=np.uint8)
    frozen = np.ascontiguousarray(np.asarray(frozen, dtype=np.int32))
    rc = lib().orc_decode_sc_float(N, K, _ptr(frozen), _ptr(x), x.shape[0], _ptr(out))
    if rc != 0:
        raise RuntimeError(f"oracle decode failed rc={rc}")
    return out


# Float-domain kinds (include/qpd.h enum qpd_kind)
FLOAT_KIND = {"SC": 0, "SCL": 7, "CA-SCL": 8, "FastSC": 9, "FastSCL": 10, "SC-Uniform": 11, "SCL-Uniform": 12,
              "SC-Lloyd": 13, "SCL-Lloyd": 14}


def decode_float(kind: str, N: int, K: int, frozen, llr, L: int = 1, node_type=None, quant=None, A: int = 0,
                 crc_n: int = 0, crc_loc=()) -> np.ndarray:
    """Restated float-domain decoder ``kind`` on float64 LLRs [B, N] -> uint8 [B, K] ([B, A] for CA-SCL).
    ``quant``: quant.UniformQuant (Uniform kinds) or quant.LloydQuant (Lloyd kinds)."""
    k = FLOAT_KIND[kind]
    x = np.ascontiguousarray(np.asarray(llr, dtype=np.float64).reshape(-1, N))
    B = x.shape[0]
    ob = A if kind == "CA-SCL" else K
    out = np.zeros((B, ob), dtype=np.uint8)
    frozen = np.ascontiguousarray(np.asarray(frozen, dtype=np.int32))
    nt = None if node_type is None else np.ascontiguousarray(np.asarray(node_type).astype(np.int32))
    loc = np.ascontiguousarray(np.asarray(crc_loc, dtype=np.int32))
    v = 0
    rf = rg = bnd = boff = blen = rec = roff = rlen = None
    if quant is not None:
        v = quant.v
        if hasattr(quant, "r_f"):
            rf, rg = quant.r_f, quant.r_g
        else:
            bnd, boff, blen, rec, roff, rlen = (quant.bnd, quant.bnd_off, quant.bnd_len, quant.rec, quant.rec_off,
                                                quant.rec_len)
    rc = lib().orc_decode_float(k, N, K, L, _ptr(frozen), _ptr(nt), v, _ptr(rf), _ptr(rg), _ptr(bnd), _ptr(boff),
                                _ptr(blen), _ptr(rec), _ptr(roff), _ptr(rlen), A, crc_n, _ptr(loc), loc.size,
                                _ptr(x), B, _ptr(out))
    if rc != 0:
        raise RuntimeError(f"oracle decode failed rc={rc}")
    return out


def reference_module():
    """The reference decoders compiled from /root/reference sources, or None."""
    hits = glob.glob(os.path.join(REF_DIR, "_refPolarDecoder*.so"))
    if not hits:
        return None
    if REF_DIR not in sys.path:
        sys.path.insert(0, REF_DIR)
    import _refPolarDecoder  # noqa: E402

    return _refPolarDecoder
