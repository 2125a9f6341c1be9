"""ctypes binding of libqpd.so (the C-ABI declared in include/qpd.h).

The library is built in-tree by :func:`quantized_decoder_polar_codes_amd.build.build_native`
(hipcc --offload-arch=gfx950).  There is no fallback: if the library is
missing, or no HIP device is present, decoding raises.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("QPD_LIB") or os.path.join(HERE, "libqpd.so")

(QPD_SC_FLOAT, QPD_SC_LUT, QPD_SCL_LUT, QPD_FASTSC_LUT, QPD_FASTSCL_LUT, QPD_CASCL_LUT, QPD_CAFASTSCL_LUT,
 QPD_SCL_FLOAT, QPD_CASCL_FLOAT, QPD_FASTSC_FLOAT, QPD_FASTSCL_FLOAT, QPD_SC_UNIFORM, QPD_SCL_UNIFORM, QPD_SC_LLOYD,
 QPD_SCL_LLOYD) = range(15)
FLOAT_KINDS = (QPD_SC_FLOAT, QPD_SCL_FLOAT, QPD_CASCL_FLOAT, QPD_FASTSC_FLOAT, QPD_FASTSCL_FLOAT, QPD_SC_UNIFORM,
               QPD_SCL_UNIFORM, QPD_SC_LLOYD, QPD_SCL_LLOYD)
ABI_VERSION = 6
QPD_ENGINE_AUTO, QPD_ENGINE_GENERIC, QPD_ENGINE_FAST = range(3)
QPD_OK, QPD_E_INVALID, QPD_E_UNSUPPORTED, QPD_E_DEVICE, QPD_E_INPUT = 0, -1, -2, -3, -4

# Every symbol include/qpd.h declares (tests check the library exports them).
EXPORTED = (
    "qpd_abi_version",
    "qpd_build_id",
    "qpd_last_error",
    "qpd_create",
    "qpd_destroy",
    "qpd_decode",
    "qpd_decode_f64",
    "qpd_decode_host",
    "qpd_decode_f64_host",
    "qpd_check_input_error",
    "qpd_get_info",
    "qpd_mc_frames",
    "qpd_mc_decode",
    "qpd_optls_quantizer",
    "qpd_lutgen_mindistortion",
    "qpd_profile",
    "qpd_kernel_times",
    "qpd_probe_lds",
    "qpd_set_host_engine",
)
QPD_KC_PRE, QPD_KC_DECODE, QPD_KC_MC, QPD_KC_PFX, QPD_KC_COUNT = range(5)
QPD_PROBE_BPERMUTE, QPD_PROBE_READ_B32, QPD_PROBE_READ_B64 = range(3)
QPD_HOST_AUTO, QPD_HOST_GPU, QPD_HOST_CPU = range(3)
QPD_RAN_NONE, QPD_RAN_GPU, QPD_RAN_HOST = range(3)

_P = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64


class QpdConfig(ctypes.Structure):
    _fields_ = [
        ("kind", _i32),
        ("N", _i32),
        ("K", _i32),
        ("L", _i32),
        ("v", _i32),
        ("frozen_bits", _P),
        ("node_type", _P),
        ("lut_f", _P),
        ("lut_f_count", _i32),
        ("f_base", _P),
        ("f_step", _i32),
        ("lut_g", _P),
        ("lut_g_count", _i32),
        ("g_base", _P),
        ("g_step", _i32),
        ("vcl", _P),
        ("vcl_rows", _i32),
        ("device", _i32),
        ("max_waves", _i32),
        ("engine", _i32),
        ("A", _i32),
        ("crc_n", _i32),
        ("crc_loc", _P),
        ("crc_loc_count", _i32),
        ("r_f", _P),
        ("r_g", _P),
        ("q_bnd", _P),
        ("q_bnd_count", _i32),
        ("q_rec", _P),
        ("q_rec_count", _i32),
        ("bnd_off", _P),
        ("bnd_len", _P),
        ("rec_off", _P),
        ("rec_len", _P),
    ]


class QpdMcChannel(ctypes.Structure):
    _fields_ = [
        ("sigma", ctypes.c_double),
        ("q", _i32),
        ("n_edges", _i32),
        ("edges", _P),
        ("lut", _P),
    ]


class QpdInfo(ctypes.Structure):
    _fields_ = [
        ("kind", _i32),
        ("N", _i32),
        ("K", _i32),
        ("L", _i32),
        ("v", _i32),
        ("num_ops", _i32),
        ("frames_per_wave", _i32),
        ("lanes_per_frame", _i32),
        ("max_waves", _i32),
        ("scratch_bytes_per_wave", _i64),
        ("engine", _i32),
        ("lds_bytes_per_wave", _i32),
        ("lds_from_depth", _i32),
        ("out_bits", _i32),
        ("host_max_frames", _i64),
        ("prefix_ops", _i32),
        ("last_engine", _i32),
        ("lookups_per_path", _i64),
        ("fast_variant", _i32),
        ("reserved0", _i32),
    ]


_lib = None


class QpdError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libqpd error {code}: {msg}")
        self.code = code


def load():
    """Load libqpd.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)"
        )
    # One HIP runtime per process: torch's wheel bundles libamdhip64.so with the
    # same SONAME as /opt/rocm's.  Loading torch first makes libqpd.so bind to
    # the runtime torch already uses (device memory and streams are shared).
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is part of the image
        pass
    L = ctypes.CDLL(LIB_PATH)
    L.qpd_abi_version.restype = ctypes.c_int
    L.qpd_last_error.restype = ctypes.c_char_p
    L.qpd_create.argtypes = [ctypes.POINTER(QpdConfig), ctypes.POINTER(_P)]
    L.qpd_create.restype = ctypes.c_int
    L.qpd_destroy.argtypes = [_P]
    L.qpd_destroy.restype = None
    L.qpd_decode.argtypes = [_P, _P, _i64, _P, _P]
    L.qpd_decode.restype = ctypes.c_int
    L.qpd_decode_f64.argtypes = [_P, _P, _i64, _P, _P]
    L.qpd_decode_f64.restype = ctypes.c_int
    L.qpd_decode_host.argtypes = [_P, _P, _i64, _P]
    L.qpd_decode_host.restype = ctypes.c_int
    L.qpd_decode_f64_host.argtypes = [_P, _P, _i64, _P]
    L.qpd_decode_f64_host.restype = ctypes.c_int
    L.qpd_check_input_error.argtypes = [_P]
    L.qpd_check_input_error.restype = ctypes.c_int
    L.qpd_get_info.argtypes = [_P, ctypes.POINTER(QpdInfo)]
    L.qpd_get_info.restype = ctypes.c_int
    L.qpd_mc_frames.argtypes = [_P, ctypes.POINTER(QpdMcChannel), ctypes.c_uint64, _i64, _i64, _P, _P, _P]
    L.qpd_mc_frames.restype = ctypes.c_int
    L.qpd_mc_decode.argtypes = [_P, ctypes.POINTER(QpdMcChannel), ctypes.c_uint64, _i64, _i64, _P, _P, _P, _P]
    L.qpd_mc_decode.restype = ctypes.c_int
    L.qpd_optls_quantizer.argtypes = [_P, _P, _i32, _i32, _i32, _P, _P, _P, _P]
    L.qpd_optls_quantizer.restype = ctypes.c_int
    L.qpd_lutgen_mindistortion.argtypes = [_i32, _i32, _P, _P, _i32, _i32, _P, _P, _P, _P]
    L.qpd_lutgen_mindistortion.restype = ctypes.c_int
    L.qpd_profile.argtypes = [_P, _i32]
    L.qpd_profile.restype = ctypes.c_int
    L.qpd_kernel_times.argtypes = [_P, _P, _P]
    L.qpd_kernel_times.restype = ctypes.c_int
    L.qpd_probe_lds.argtypes = [_i32, _i32, ctypes.POINTER(ctypes.c_double)]
    L.qpd_probe_lds.restype = ctypes.c_int
    L.qpd_set_host_engine.argtypes = [_P, _i32]
    L.qpd_set_host_engine.restype = ctypes.c_int
    if L.qpd_abi_version() != ABI_VERSION:
        raise ImportError("libqpd.so ABI version mismatch")
    L.qpd_build_id.restype = ctypes.c_char_p
    check_build_id(L)
    _lib = L
    return L


def check_build_id(L) -> None:
    """The in-tree library must be built from the sources next to it (build.py
    stamps their hash into it): a stale binary raises instead of running.
    QPD_LIB (an explicitly chosen diagnostic build) skips the check."""
    if os.environ.get("QPD_LIB"):
        return
    from . import build

    if not os.path.isdir(build.SRC):  # a library shipped without its sources
        return
    have, want = L.qpd_build_id().decode(), build.source_hash()
    if have != want:
        raise ImportError(f"{LIB_PATH} was built from other sources (build id {have}, tree {want}): rebuild it "
                          "with `python -c 'import __graft_entry__ as g; g.build()'`")


def check(rc: int) -> None:
    if rc == QPD_OK:
        return
    msg = load().qpd_last_error().decode(errors="replace")
    if rc in (QPD_E_INVALID, QPD_E_UNSUPPORTED, QPD_E_INPUT):
        raise ValueError(msg)
    raise QpdError(rc, msg)
