"""MinDistortion LUT design: the reference's offline
generator (GenerateLookUpTable_LLRDomain.py:9-73) without OpenCV, on the
native code in csrc/qpd_lutgen.cpp (multi-threaded over the nodes of a level).

* :func:`optls_quantizer` -- LLRQuantizer::find_OptLS_quantizer
  (LLRQuantizer.cpp:67-165; Python twin MinDistortionQuantizer.py:28-99).
* :func:`channel_quantizer` -- the physical-channel quantizer the drivers build
  per Eb/N0 (mainQuantizedDecoder_LLRDomain.py:135-145): 128 uniform bins of
  the two-Gaussian LLR density merged to ``q`` symbols.
* :func:`mindistortion_luts` -- LLRQuantizerSC.run
  (QLLRDensityEvolution_MinDistortion.py:73-126).
* :func:`design` -- the whole script: channel quantizer at the design SNR,
  then the decoder tables; returns the reference's dict/list formats and a
  :class:`~quantized_decoder_polar_codes_amd.lut.PackedLUT`.
* :func:`save_npz` / :func:`load_npz` -- the on-disk format here (plain
  arrays, no pickle).  :func:`write_reference_pickles` writes the files the
  reference drivers load (``LUT_F_SNRdB={:.0f}.pkl`` ...,
  mainQuantizedDecoder_LLRDomain.py:76-84); reading pickles back is left to
  the caller, for files they generated themselves.

``sum_order="cpp"`` (default) sums inside the DP sequentially, like the C++
quantizer the reference generator calls; ``"numpy"`` uses numpy's pairwise
sums, like the reference's Python twin -- the form the tests pin against the
reference code (the OpenCV build is unavailable here).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

from . import _lib
from .codes import channel_llr_density_table
from .lut import PackedLUT, pack_luts

_ORDER = {"cpp": 0, "numpy": 1}


def _p(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def optls_quantizer(density, quanta, K: int, sum_order: str = "cpp"):
    """Merge M quanta into K (minimum squared error over sorted groups).
    Returns (density[K], quanta[K], lut[M] int32, distortion)."""
    d = np.ascontiguousarray(np.asarray(density, dtype=np.float64).reshape(-1))
    q = np.ascontiguousarray(np.asarray(quanta, dtype=np.float64).reshape(-1))
    M = d.size
    if q.size != M or not 1 <= K <= M:
        raise ValueError(f"need len(density) == len(quanta) >= K, got {M}, {q.size}, K={K}")
    od, oq = np.zeros(K), np.zeros(K)
    lut = np.zeros(M, dtype=np.int32)
    dist = ctypes.c_double()
    rc = _lib.load().qpd_optls_quantizer(_p(d), _p(q), M, K, _ORDER[sum_order], _p(od), _p(oq), _p(lut),
                                         ctypes.byref(dist))
    if rc:
        raise ValueError("qpd_optls_quantizer rejected its arguments")
    return od, oq, lut, dist.value


def channel_quantizer(sigma: float, q_uniform: int = 128, q: int = 16, sum_order: str = "cpp"):
    """The drivers' channel quantizer for AWGN std ``sigma``
    (mainQuantizedDecoder_LLRDomain.py:135-145; GenerateLookUpTable_LLRDomain.py:40-52).
    Returns (density[q], quanta[q], interval_x[q_uniform+1], channel_lut[q_uniform])."""
    e_llr = 2 / sigma ** 2
    d_llr = np.sqrt(2 * e_llr)
    hi, lo = e_llr + 3 * d_llr, -e_llr - 3 * d_llr
    pyx, interval_x, quanta = channel_llr_density_table(q_uniform, lo, hi, e_llr, -e_llr, d_llr)
    dens, qu, lut, _ = optls_quantizer(pyx, quanta, q, sum_order)
    return dens, qu, interval_x, lut


def mindistortion_luts(N: int, v: int, channel_density, channel_quanta, sum_order: str = "cpp", threads: int = 0):
    """Density evolution + per-node DP merge.  Returns dict with lut_f uint8
    [N-1, v, v], lut_g uint8 [N-1, 2, v, v], llr_density / llr_quanta float64
    [log2 N + 1, N, v] (llr_quanta is the decoders' virtual_channel_llr)."""
    n = int(np.log2(N))
    if N < 2 or (1 << n) != N:
        raise ValueError("N must be a power of two >= 2")
    cd = np.ascontiguousarray(np.asarray(channel_density, dtype=np.float64).reshape(-1))
    cq = np.ascontiguousarray(np.asarray(channel_quanta, dtype=np.float64).reshape(-1))
    if cd.size != v or cq.size != v:
        raise ValueError(f"channel density/quanta must have v={v} entries")
    lut_f = np.zeros((N - 1, v, v), dtype=np.uint8)
    lut_g = np.zeros((N - 1, 2, v, v), dtype=np.uint8)
    dens = np.zeros((n + 1, N, v))
    quan = np.zeros((n + 1, N, v))
    rc = _lib.load().qpd_lutgen_mindistortion(N, v, _p(cd), _p(cq), _ORDER[sum_order], int(threads), _p(lut_f),
                                              _p(lut_g), _p(dens), _p(quan))
    if rc == -2:
        raise ValueError("a node has fewer distinct LLR values than v (the reference aborts: CV_Assert(M >= K))")
    if rc:
        raise ValueError("qpd_lutgen_mindistortion rejected its arguments")
    return {"lut_f": lut_f, "lut_g": lut_g, "llr_density": dens, "llr_quanta": quan}


@dataclass
class LutDesign:
    N: int
    v: int
    design_snr_db: float
    lut_f: np.ndarray          # uint8 [N-1, v, v]
    lut_g: np.ndarray          # uint8 [N-1, 2, v, v]
    llr_quanta: np.ndarray     # [n+1, N, v] (virtual_channel_llr)
    llr_density: np.ndarray    # [n+1, N, v]
    channel_density: np.ndarray
    channel_quanta: np.ndarray

    def packed(self) -> PackedLUT:
        """Tables in the decoders' packed form (one table per node)."""
        return pack_luts(self.N, self.lut_f, self.lut_g, self.llr_quanta)

    def reference_dicts(self):
        """The generator's own output format: {node_posi: [table] * (N >> (depth+1))}
        for f and g (GenerateLookUpTable_LLRDomain.py:56-60)."""
        fs, gs = {}, {}
        for p in range(self.N - 1):
            depth = int(np.log2(p + 1))
            reps = self.N >> (depth + 1)
            fs[p] = [self.lut_f[p].astype(np.int32)] * reps
            gs[p] = [self.lut_g[p].astype(np.int32)] * reps
        return fs, gs


def design(N: int, v: int = 16, design_snr_db: float = 3.0, q_channel_uniform: int = 128, q_channel: int | None = None,
           sum_order: str = "cpp", threads: int = 0) -> LutDesign:
    """GenerateLookUpTable_LLRDomain.py:9-73 (sigma = sqrt(1 / DesignSNR), :36-37)."""
    q_channel = v if q_channel is None else q_channel
    if q_channel != v:
        raise ValueError("the decoder alphabet is the channel alphabet: q_channel must equal v")
    sigma = float(np.sqrt(1 / 10 ** (design_snr_db / 10)))
    cd, cq, _, _ = channel_quantizer(sigma, q_channel_uniform, q_channel, sum_order)
    t = mindistortion_luts(N, v, cd, cq, sum_order, threads)
    return LutDesign(N, v, design_snr_db, t["lut_f"], t["lut_g"], t["llr_quanta"], t["llr_density"], cd, cq)


def save_npz(path: str, d: LutDesign) -> None:
    np.savez_compressed(path, N=d.N, v=d.v, design_snr_db=d.design_snr_db, lut_f=d.lut_f, lut_g=d.lut_g,
                        llr_quanta=d.llr_quanta, llr_density=d.llr_density, channel_density=d.channel_density,
                        channel_quanta=d.channel_quanta)


def load_npz(path: str) -> LutDesign:
    z = np.load(path, allow_pickle=False)
    return LutDesign(int(z["N"]), int(z["v"]), float(z["design_snr_db"]), z["lut_f"], z["lut_g"], z["llr_quanta"],
                     z["llr_density"], z["channel_density"], z["channel_quanta"])


def write_reference_pickles(save_dir: str, d: LutDesign) -> list:
    """The four files GenerateLookUpTable_LLRDomain.py:62-73 writes, loadable by
    the reference drivers unchanged."""
    import pickle

    os.makedirs(save_dir, exist_ok=True)
    fs, gs = d.reference_dicts()
    paths = []
    for name, obj in (("LUT_F", fs), ("LUT_G", gs), ("LLRQuanta", d.llr_quanta), ("LLRDensity", d.llr_density)):
        p = os.path.join(save_dir, "{:s}_SNRdB={:.0f}.pkl".format(name, d.design_snr_db))
        with open(p, "wb") as f:
            pickle.dump(obj, f)
        paths.append(p)
    return paths
