"""Host-side mirror of the reference's pybind11 decoder classes -- all 15 of
_libPolarDecoder.cpp:29-50.

Same class names, positional order, keyword names and ``decode`` argument as
the reference (py_interface/py_SCLUTDecoder.cpp:11-14, py_SCLLUTDecoder.cpp:12-15,
py_FastSCLUTDecoder.cpp:12-15, py_FastSCLLUTDecoder.cpp:13-16,
py_SCDecoder.cpp:10-12, py_SCLDecoder.cpp:10-12, py_CASCLDecoder.cpp:10-13,
py_FastSCDecoder.cpp:11-14, py_FastSCLDecoder.cpp:10-13,
py_SCUniformDecoder.cpp:10-14, py_SCLUniformQuantizedDecoder.cpp:10-14,
py_SCLloydQuantizedDecoder.cpp:10-15, py_SCLLloydQuantizedDecoder.cpp:10-15):
``decode`` takes one frame and returns a new ``numpy.ndarray`` of dtype uint8
and length K (A for the CRC-aided classes).  Every decode runs in libqpd.so:
batches on the GPU kernels, the few frames of a per-frame call on its host
engine (qpd_decode_host; a GPU call costs ~0.1 ms before decoding anything,
the reference's SC-LUT call ~10 us).  The package fails to load without the
library and a decoder cannot be created without a HIP device.

Additions (not in the reference): ``decode_batch(x[B, N])`` for throughput
(numpy in -> numpy out; a torch CUDA tensor in -> torch CUDA tensor out,
asynchronous on torch's current stream), and validation with ``ValueError``
where the reference has undefined behaviour.
"""
from __future__ import annotations

import ctypes
import threading

import numpy as np

from . import _lib
from .lut import PackedLUT, pack_luts
from .quant import LloydQuant, UniformQuant, pack_lloyd, pack_uniform

__all__ = ["SCDecoder", "SCLUTDecoder", "SCLLUTDecoder", "FastSCLUTDecoder", "FastSCLLUTDecoder",
           "CASCLLUTDecoder", "CAFastSCLLUTDecoder", "SCLDecoder", "CASCLDecoder", "FastSCDecoder", "FastSCLDecoder",
           "SCUniformQuantizedDecoder", "SCLUniformQuantizedDecoder", "SCLloydQuantizedDecoder",
           "SCLLloydQuantizedDecoder"]

# The CRC the reference CA decoders actually check (CASCLLUTDecoder.h:33-34,
# CAFastSCLLUTDecoder.h:29-30): CRC-24 with these coefficient indices, whatever
# crc_n / crc_p the CASCLLUTDecoder constructor receives (decode never reads them).
CRC24_LOC = (24, 23, 21, 20, 17, 15, 13, 12, 8, 4, 2, 1, 0)


def _as_i32(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x).astype(np.int32))


def _ptr(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def _torch():
    try:
        import torch  # noqa: F401

        return torch
    except Exception:  # pragma: no cover - torch is part of the image
        return None


class _DecoderBase:
    _kind: int = -1

    @property
    def _float_input(self) -> bool:
        return self._kind in _lib.FLOAT_KINDS

    def __init__(self, N, K, L, frozen_bits, message_bits, node_type, packed: PackedLUT | None, device=None,
                 max_waves: int = 0, engine: str = "auto", A: int | None = None, crc_n: int = 24,
                 crc_loc=CRC24_LOC, quant: UniformQuant | LloydQuant | None = None, create: bool = True):
        self.N = int(N)
        self.K = int(K)
        self.L = int(L)
        self.A = self.K if A is None else int(A)
        self.out_bits = self.A
        frozen = _as_i32(frozen_bits).reshape(-1)
        if frozen.size != self.N:
            raise ValueError(f"frozen_bits must have N={self.N} entries, got {frozen.size}")
        self.frozen_bits = frozen
        # message_bits is stored but never read by the reference
        self.message_bits = np.asarray(message_bits)
        self.node_type = None if node_type is None else _as_i32(node_type).reshape(-1)
        if self.node_type is not None and self.node_type.size != 2 * self.N - 1:
            raise ValueError(f"node_type must have 2N-1={2 * self.N - 1} entries, got {self.node_type.size}")
        self.packed = packed
        cfg = _lib.QpdConfig()
        cfg.kind = self._kind
        cfg.N, cfg.K, cfg.L = self.N, self.K, self.L
        cfg.frozen_bits = _ptr(self.frozen_bits)
        cfg.node_type = _ptr(self.node_type)
        if packed is not None:
            if packed.N != self.N:
                raise ValueError(f"tables are for N={packed.N}, decoder N={self.N}")
            cfg.v = packed.v
            cfg.lut_f, cfg.lut_f_count = _ptr(packed.lut_f), packed.lut_f.shape[0]
            cfg.f_base, cfg.f_step = _ptr(packed.f_base), packed.f_step
            cfg.lut_g, cfg.lut_g_count = _ptr(packed.lut_g), packed.lut_g.shape[0]
            cfg.g_base, cfg.g_step = _ptr(packed.g_base), packed.g_step
            cfg.vcl, cfg.vcl_rows = _ptr(packed.vcl), packed.vcl_rows
        if device is None:
            torch = _torch()
            device = torch.cuda.current_device() if torch is not None and torch.cuda.is_available() else -1
        self.device = int(device)
        cfg.device = self.device
        cfg.max_waves = int(max_waves)
        cfg.engine = {"auto": _lib.QPD_ENGINE_AUTO, "generic": _lib.QPD_ENGINE_GENERIC,
                      "fast": _lib.QPD_ENGINE_FAST}[engine]
        self.quant = quant
        if isinstance(quant, UniformQuant):
            cfg.v = quant.v
            cfg.r_f, cfg.r_g = _ptr(quant.r_f), _ptr(quant.r_g)
        elif isinstance(quant, LloydQuant):
            cfg.v = quant.v
            cfg.q_bnd, cfg.q_bnd_count = _ptr(quant.bnd), quant.bnd.size
            cfg.q_rec, cfg.q_rec_count = _ptr(quant.rec), quant.rec.size
            cfg.bnd_off, cfg.bnd_len = _ptr(quant.bnd_off), _ptr(quant.bnd_len)
            cfg.rec_off, cfg.rec_len = _ptr(quant.rec_off), _ptr(quant.rec_len)
        self._crc_loc = np.ascontiguousarray(np.asarray(crc_loc, dtype=np.int32))
        if self._kind in (_lib.QPD_CASCL_LUT, _lib.QPD_CAFASTSCL_LUT, _lib.QPD_CASCL_FLOAT):
            cfg.A, cfg.crc_n = self.A, int(crc_n)
            cfg.crc_loc, cfg.crc_loc_count = _ptr(self._crc_loc), self._crc_loc.size
        self._cfg = cfg  # the arrays it points to are attributes of self
        if not create:  # configuration only (tests of the host engine on CPU): no device decoder
            self._h = None
            return
        h = ctypes.c_void_p()
        lib = _lib.load()
        _lib.check(lib.qpd_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        # the per-frame call's own buffers and bound entry point (numpy's
        # pointer extraction costs ~2 us per array, as much as a whole SC-LUT
        # frame on the host engine): decode() copies into / out of them
        self._one_in = np.empty(self.N, dtype=np.float64 if self._float_input else np.int32)
        self._one_out = np.empty(self.out_bits, dtype=np.uint8)
        self._one_args = (ctypes.c_void_p(self._one_in.ctypes.data), ctypes.c_void_p(self._one_out.ctypes.data))
        self._one_fn = lib.qpd_decode_f64_host if self._float_input else lib.qpd_decode_host
        self._one_lock = threading.Lock()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _lib.load().qpd_destroy(h)
            except Exception:
                pass
            self._h = None

    # -- introspection ---------------------------------------------------------
    def info(self) -> dict:
        inf = _lib.QpdInfo()
        _lib.check(_lib.load().qpd_get_info(self._h, ctypes.byref(inf)))
        return {k: getattr(inf, k) for k, _ in inf._fields_}

    def profile(self, enable: bool = True) -> None:
        """Bracket every kernel launch of this decoder with HIP events on its
        stream (qpd_profile); read the sums with :meth:`kernel_times`."""
        _lib.check(_lib.load().qpd_profile(self._h, int(bool(enable))))

    def kernel_times(self) -> dict:
        """{class: (ms summed, launches)} since the last call, for the classes
        'pre' (root pre-pass), 'decode', 'mc' (frame generator) and 'pfx'
        (frozen prefix, lut_prefix_kernel)."""
        ms = (ctypes.c_double * _lib.QPD_KC_COUNT)()
        n = (ctypes.c_int64 * _lib.QPD_KC_COUNT)()
        _lib.check(_lib.load().qpd_kernel_times(self._h, ms, n))
        return {name: (ms[i], n[i]) for i, name in enumerate(("pre", "decode", "mc", "pfx"))}

    # -- decoding --------------------------------------------------------------
    def decode_batch(self, x):
        """Decode B frames.  numpy [B, N] -> numpy uint8 [B, K] (synchronous);
        torch CUDA tensor [B, N] -> torch CUDA uint8 [B, K] on the current stream.
        (A instead of K for the CRC-aided decoders.)"""
        torch = _torch()
        lib = _lib.load()
        if torch is not None and isinstance(x, torch.Tensor) and x.is_cuda:
            want = torch.float64 if self._float_input else torch.int32
            xs = x.reshape(-1, self.N).to(want).contiguous()
            B = xs.shape[0]
            out = torch.empty((B, self.out_bits), dtype=torch.uint8, device=xs.device)
            stream = torch.cuda.current_stream(xs.device).cuda_stream
            fn = lib.qpd_decode_f64 if self._float_input else lib.qpd_decode
            _lib.check(fn(self._h, ctypes.c_void_p(xs.data_ptr()), B, ctypes.c_void_p(out.data_ptr()),
                          ctypes.c_void_p(stream)))
            return out
        if torch is not None and isinstance(x, torch.Tensor):
            x = x.numpy()
        a = np.asarray(x)
        a = np.ascontiguousarray(a.astype(np.float64 if self._float_input else np.int32).reshape(-1, self.N))
        B = a.shape[0]
        out = np.empty((B, self.out_bits), dtype=np.uint8)
        fn = lib.qpd_decode_f64_host if self._float_input else lib.qpd_decode_host
        _lib.check(fn(self._h, _ptr(a), B, _ptr(out)))
        return out

    def set_host_engine(self, mode: str = "auto") -> None:
        """Where host-buffer calls (``decode``, numpy ``decode_batch``) run:
        "auto" (the host engine for the few frames a per-frame call brings, the
        GPU for batches; ``info()["host_max_frames"]``), "gpu" or "cpu"."""
        m = {"auto": _lib.QPD_HOST_AUTO, "gpu": _lib.QPD_HOST_GPU, "cpu": _lib.QPD_HOST_CPU}[mode]
        _lib.check(_lib.load().qpd_set_host_engine(self._h, m))

    def _decode_one(self, x) -> np.ndarray:
        # the per-frame call (mainQuantizedDecoder_LLRDomain.py:178): one frame
        # straight to the host-buffer entry point, no batch reshaping; the
        # values are force-cast as pybind11's array_t<int> / <double> does
        a = np.asarray(x).reshape(-1)
        if a.size < self.N:
            raise ValueError(f"decode expects N={self.N} values, got {a.size}")
        with self._one_lock:  # the GIL is released during the call: keep the buffers per call
            np.copyto(self._one_in, a[: self.N], casting="unsafe")
            _lib.check(self._one_fn(self._h, self._one_args[0], 1, self._one_args[1]))
            return self._one_out.copy()


class _LUTDecoder(_DecoderBase):
    def decode(self, channel_quantized_symbols):
        return self._decode_one(channel_quantized_symbols)


class SCLUTDecoder(_LUTDecoder):
    """SC-LUT (SCLUTDecoder.cpp:21-124)."""

    _kind = _lib.QPD_SC_LUT

    def __init__(self, N, K, frozen_bits, message_bits, LUT_f, LUT_g, virtual_channel_llr, **kw):
        super().__init__(N, K, 1, frozen_bits, message_bits, None, pack_luts(int(N), LUT_f, LUT_g, virtual_channel_llr),
                         **kw)


class SCLLUTDecoder(_LUTDecoder):
    """SCL-LUT (SCLLUTDecoder.cpp:47-253)."""

    _kind = _lib.QPD_SCL_LUT

    def __init__(self, N, K, L, frozen_bits, message_bits, LUT_f, LUT_g, virtual_channel_llr, **kw):
        super().__init__(N, K, L, frozen_bits, message_bits, None, pack_luts(int(N), LUT_f, LUT_g, virtual_channel_llr),
                         **kw)


class FastSCLUTDecoder(_DecoderBase):
    """FastSC-LUT (FastSCLUT.cpp:27-206); note the reference's kwargs LUT_Fs/LUT_Gs
    and decode(llr) (py_FastSCLUTDecoder.cpp:12-15)."""

    _kind = _lib.QPD_FASTSC_LUT

    def __init__(self, N, K, frozen_bits, message_bits, node_type, LUT_Fs, LUT_Gs, virtual_channel_llr, **kw):
        super().__init__(N, K, 1, frozen_bits, message_bits, node_type,
                         pack_luts(int(N), LUT_Fs, LUT_Gs, virtual_channel_llr), **kw)

    def decode(self, llr):
        return self._decode_one(llr)


class FastSCLLUTDecoder(_LUTDecoder):
    """FastSCL-LUT (FastSCLLUTDecoder.cpp:57-408)."""

    _kind = _lib.QPD_FASTSCL_LUT

    def __init__(self, N, K, L, frozen_bits, message_bits, node_type, LUT_f, LUT_g, virtual_channel_llr, **kw):
        super().__init__(N, K, L, frozen_bits, message_bits, node_type,
                         pack_luts(int(N), LUT_f, LUT_g, virtual_channel_llr), **kw)


class CASCLLUTDecoder(_LUTDecoder):
    """CRC-aided SCL-LUT (CASCLLUTDecoder.cpp:64-303; ctor py_CASCLLUTDecoder.cpp:10-17).
    ``decode`` returns the A message bits.  Like the reference, ``crc_n``/``crc_p``
    are accepted and stored but the check is always CRC-24 (CRC24_LOC)."""

    _kind = _lib.QPD_CASCL_LUT

    def __init__(self, N, K, A, L, frozen_bits, message_bits, crc_n, crc_p, LUT_f, LUT_g, virtual_channel_llr, **kw):
        self.crc_n, self.crc_p = crc_n, crc_p
        super().__init__(N, K, L, frozen_bits, message_bits, None, pack_luts(int(N), LUT_f, LUT_g, virtual_channel_llr),
                         A=A, **kw)


class CAFastSCLLUTDecoder(_LUTDecoder):
    """CRC-aided FastSCL-LUT (CAFastSCLLUTDecoder.cpp:58-454; ctor
    py_CAFastSCLLUTDecoder.cpp:10-16).  ``decode`` returns the A message bits."""

    _kind = _lib.QPD_CAFASTSCL_LUT

    def __init__(self, N, K, A, L, frozen_bits, message_bits, node_type, LUT_f, LUT_g, virtual_channel_llr, **kw):
        super().__init__(N, K, L, frozen_bits, message_bits, node_type,
                         pack_luts(int(N), LUT_f, LUT_g, virtual_channel_llr), A=A, **kw)


class SCDecoder(_DecoderBase):
    """Float SC, min-sum on float64 LLRs (SCDecoder.cpp:14-89)."""

    _kind = _lib.QPD_SC_FLOAT

    def __init__(self, N, K, frozen_bits, message_bits, **kw):
        super().__init__(N, K, 1, frozen_bits, message_bits, None, None, **kw)

    def decode(self, llr):
        return self._decode_one(llr)


class _FloatDecoder(_DecoderBase):
    def decode(self, llr):
        return self._decode_one(llr)


class SCLDecoder(_FloatDecoder):
    """Float SCL, min-sum list decoding on float64 LLRs (SCLDecoder.cpp:38-176)."""

    _kind = _lib.QPD_SCL_FLOAT

    def __init__(self, N, K, L, frozen_bits, message_bits, **kw):
        super().__init__(N, K, L, frozen_bits, message_bits, None, None, **kw)


class CASCLDecoder(_FloatDecoder):
    """CRC-aided float SCL (CASCLDecoder.cpp:74-249; ctor py_CASCLDecoder.cpp:10-12).
    Unlike the CA-LUT classes it checks the CRC it is given: ``crc_n`` bits with
    divisor coefficients ``crc_p`` (a list of indices, CASCLDecoder.cpp:49-53).
    ``decode`` returns the A message bits."""

    _kind = _lib.QPD_CASCL_FLOAT

    def __init__(self, N, K, A, L, frozen_bits, message_bits, crc_n, crc_p, **kw):
        self.crc_n, self.crc_p = int(crc_n), list(crc_p)
        super().__init__(N, K, L, frozen_bits, message_bits, None, None, A=A, crc_n=int(crc_n), crc_loc=crc_p, **kw)


class FastSCDecoder(_FloatDecoder):
    """Float Fast-SC with R0/R1/REP/SPC nodes (FastSCDecoder.cpp:21-174)."""

    _kind = _lib.QPD_FASTSC_FLOAT

    def __init__(self, N, K, frozen_bits, message_bits, node_type, **kw):
        super().__init__(N, K, 1, frozen_bits, message_bits, node_type, None, **kw)


class FastSCLDecoder(_FloatDecoder):
    """Float Fast-SCL with R0/R1/REP nodes, no SPC (FastSCLDecoder.cpp:49-423)."""

    _kind = _lib.QPD_FASTSCL_FLOAT

    def __init__(self, N, K, L, frozen_bits, message_bits, node_type, **kw):
        super().__init__(N, K, L, frozen_bits, message_bits, node_type, None, **kw)


class SCUniformQuantizedDecoder(_FloatDecoder):
    """SC with uniform re-quantization after every f/g (SCUniformQuantizedDecoder.cpp:20-99)."""

    _kind = _lib.QPD_SC_UNIFORM

    def __init__(self, N, K, frozen_bits, message_bits, decoder_r_f, decoder_r_g, v, **kw):
        super().__init__(N, K, 1, frozen_bits, message_bits, None, None,
                         quant=pack_uniform(int(N), decoder_r_f, decoder_r_g, int(v)), **kw)


class SCLUniformQuantizedDecoder(_FloatDecoder):
    """SCL with uniform re-quantization (SCLUniformQuantizedDecoder.cpp:43-184)."""

    _kind = _lib.QPD_SCL_UNIFORM

    def __init__(self, N, K, L, frozen_bits, message_bits, decoder_r_f, decoder_r_g, v, **kw):
        super().__init__(N, K, L, frozen_bits, message_bits, None, None,
                         quant=pack_uniform(int(N), decoder_r_f, decoder_r_g, int(v)), **kw)


class SCLloydQuantizedDecoder(_FloatDecoder):
    """SC with Lloyd re-quantization after every f/g (SCLloydQuantizedDecoder.cpp:22-101)."""

    _kind = _lib.QPD_SC_LLOYD

    def __init__(self, N, K, frozen_bits, message_bits, boundaries_f, boundaries_g, reconstruction_f,
                 reconstruction_g, v, **kw):
        super().__init__(N, K, 1, frozen_bits, message_bits, None, None,
                         quant=pack_lloyd(int(N), boundaries_f, boundaries_g, reconstruction_f, reconstruction_g,
                                          int(v)), **kw)


class SCLLloydQuantizedDecoder(_FloatDecoder):
    """SCL with Lloyd re-quantization (SCLLloydQuantizedDecoder.cpp:46-187)."""

    _kind = _lib.QPD_SCL_LLOYD

    def __init__(self, N, K, L, frozen_bits, message_bits, boundaries_f, boundaries_g, reconstruction_f,
                 reconstruction_g, v, **kw):
        super().__init__(N, K, L, frozen_bits, message_bits, None, None,
                         quant=pack_lloyd(int(N), boundaries_f, boundaries_g, reconstruction_f, reconstruction_g,
                                          int(v)), **kw)


FLOAT_CLASSES = {"SC": SCDecoder, "SCL": SCLDecoder, "CA-SCL": CASCLDecoder, "FastSC": FastSCDecoder,
                 "FastSCL": FastSCLDecoder, "SC-Uniform": SCUniformQuantizedDecoder,
                 "SCL-Uniform": SCLUniformQuantizedDecoder, "SC-Lloyd": SCLloydQuantizedDecoder,
                 "SCL-Lloyd": SCLLloydQuantizedDecoder}


def from_quant(kind: str, N: int, K: int, frozen_bits, L: int = 1, node_type=None, quant=None, **kw):
    """Build a float-domain decoder (kind as oracle.FLOAT_KIND) from packed re-quantizers."""
    cls = FLOAT_CLASSES[kind]
    obj = cls.__new__(cls)
    lst = kind in ("SCL", "CA-SCL", "FastSCL", "SCL-Uniform", "SCL-Lloyd")
    _DecoderBase.__init__(obj, N, K, L if lst else 1, frozen_bits, 1 - np.asarray(frozen_bits), node_type, None,
                          quant=quant, **kw)
    return obj


def from_packed(kind: str, packed: PackedLUT, K: int, frozen_bits, L: int = 1, node_type=None, **kw):
    """Build a decoder directly from packed tables (skips the nested-list path)."""
    cls = {"SC-LUT": SCLUTDecoder, "SCL-LUT": SCLLUTDecoder, "FastSC-LUT": FastSCLUTDecoder,
           "FastSCL-LUT": FastSCLLUTDecoder, "CA-SCL-LUT": CASCLLUTDecoder,
           "CA-FastSCL-LUT": CAFastSCLLUTDecoder}[kind]
    obj = cls.__new__(cls)
    lst = kind in ("SCL-LUT", "FastSCL-LUT", "CA-SCL-LUT", "CA-FastSCL-LUT")
    _DecoderBase.__init__(obj, packed.N, K, L if lst else 1, frozen_bits, 1 - np.asarray(frozen_bits), node_type, packed,
                          **kw)
    return obj
