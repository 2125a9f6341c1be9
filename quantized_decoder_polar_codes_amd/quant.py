"""Decoder re-quantizers of the float-domain quantized decoders -> the packed
arrays of the C-ABI (include/qpd.h, ``qpd_config.r_f`` ... ``rec_len``).

Reference inputs:

* uniform (``SCUniformQuantizedDecoder`` / ``SCLUniformQuantizedDecoder``,
  py_SCUniformDecoder.cpp:10-14): ``decoder_r_f``, ``decoder_r_g`` -- one step
  ``r`` per node_posi (N-1 each), plus the alphabet size ``v``.  After every f/g
  the value is mapped by ``Q(x, r, M)`` (utils.cpp:8-10) with
  ``M = double(v/2 - 0.5) * r_f`` for f and ``double(v/2 - 1) * r_g`` for g
  (SCUniformQuantizedDecoder.cpp:55-56, 71-72).
* Lloyd (``SCLloydQuantizedDecoder`` / ``SCLLloydQuantizedDecoder``,
  py_SCLloydQuantizedDecoder.cpp:10-15): ``boundaries_f/g`` and
  ``reconstruction_f/g`` -- per node_posi a boundary list and a reconstruction
  list (the reference generator, QLLRDensityEvolution_Lloyd.py:17-20, writes
  ``[N-1, v+1]`` boundaries starting at -inf and ending at +inf and ``[N-1, v]``
  reconstructions).  After every f/g the value becomes
  ``reconstruct[bisect_left(boundary, x) - 1]`` (utils.cpp:12-24).

Packed Lloyd layout: table t (0 = f, 1 = g) of node p is
``bnd[bnd_off[t*(N-1)+p] : +bnd_len[...]]`` and likewise ``rec``; ragged lists
are accepted.

The quantizer *design* tools of the reference (LLRLSUniformQuantizer,
LLRLloydGA: offline, scipy integration) are out of scope (SURVEY.md §2 rows
15-17); :func:`ga_uniform` and :func:`ga_lloyd` below are simple Gaussian-
approximation designs for tests and benchmarks, not restatements.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


def _log2(N: int) -> int:
    n = int(N).bit_length() - 1
    if N < 2 or (1 << n) != N:
        raise ValueError(f"N must be a power of two >= 2, got {N}")
    return n


@dataclass
class UniformQuant:
    N: int
    v: int
    r_f: np.ndarray  # float64 [N-1]
    r_g: np.ndarray  # float64 [N-1]


@dataclass
class LloydQuant:
    N: int
    v: int
    bnd: np.ndarray  # float64, concatenated boundary lists
    bnd_off: np.ndarray  # int32 [2*(N-1)]
    bnd_len: np.ndarray  # int32 [2*(N-1)]
    rec: np.ndarray  # float64, concatenated reconstruction lists
    rec_off: np.ndarray  # int32 [2*(N-1)]
    rec_len: np.ndarray  # int32 [2*(N-1)]


def pack_uniform(N: int, decoder_r_f, decoder_r_g, v: int) -> UniformQuant:
    """The reference's ``decoder_r_f`` / ``decoder_r_g`` (lists or arrays of N-1 steps)."""
    _log2(int(N))
    rf = np.ascontiguousarray(np.asarray(decoder_r_f, dtype=np.float64).reshape(-1))
    rg = np.ascontiguousarray(np.asarray(decoder_r_g, dtype=np.float64).reshape(-1))
    if rf.size < N - 1 or rg.size < N - 1:
        raise ValueError(f"decoder_r_f / decoder_r_g need N-1={N - 1} entries, got {rf.size} / {rg.size}")
    return UniformQuant(int(N), int(v), rf[: N - 1].copy(), rg[: N - 1].copy())


def _rows(x, N: int, what: str):
    if isinstance(x, np.ndarray) and x.dtype != object:
        if x.ndim != 2:
            raise ValueError(f"{what}: expected a [N-1, m] array, got shape {x.shape}")
        rows = list(x)
    else:
        rows = list(x)
    if len(rows) < N - 1:
        raise ValueError(f"{what}: need N-1={N - 1} per-node lists, got {len(rows)}")
    return [np.asarray(r, dtype=np.float64).reshape(-1) for r in rows[: N - 1]]


def pack_lloyd(N: int, boundaries_f, boundaries_g, reconstruction_f, reconstruction_g, v: int) -> LloydQuant:
    """The reference's per-node Lloyd boundary / reconstruction lists."""
    _log2(int(N))
    parts_b, parts_r = [], []
    boff, blen, roff, rlen = [], [], [], []
    nb = nr = 0
    for tb, tr, what in ((boundaries_f, reconstruction_f, "f"), (boundaries_g, reconstruction_g, "g")):
        B = _rows(tb, N, f"boundaries_{what}")
        R = _rows(tr, N, f"reconstruction_{what}")
        for b, r in zip(B, R):
            if b.size == 0 or r.size == 0:
                raise ValueError("empty boundary / reconstruction list")
            boff.append(nb)
            blen.append(b.size)
            roff.append(nr)
            rlen.append(r.size)
            parts_b.append(b)
            parts_r.append(r)
            nb += b.size
            nr += r.size
    i32 = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.int32))  # noqa: E731
    return LloydQuant(int(N), int(v), np.ascontiguousarray(np.concatenate(parts_b)), i32(boff), i32(blen),
                      np.ascontiguousarray(np.concatenate(parts_r)), i32(roff), i32(rlen))


# ---------------------------------------------------------------------------
# Gaussian-approximation designs (tests / benchmarks)
# ---------------------------------------------------------------------------
def _phi(x):
    x = np.asarray(x, dtype=np.float64)
    return np.where(x < 10, np.exp(-0.4527 * np.power(np.maximum(x, 1e-12), 0.86) + 0.0218),
                    np.sqrt(np.pi / np.maximum(x, 1e-12)) * np.exp(-x / 4) * (1 - 10 / (7 * np.maximum(x, 1e-12))))


def _phi_inv(y: float) -> float:
    lo, hi = 1e-9, 1e4
    for _ in range(200):
        mid = 0.5 * (lo + hi)
        if _phi(mid) > y:
            lo = mid
        else:
            hi = mid
    return 0.5 * (lo + hi)


def ga_means(N: int, sigma: float):
    """Per-node GA means of the f and g outputs (node_posi order)."""
    n = _log2(N)
    mu_f = np.zeros(N - 1)
    mu_g = np.zeros(N - 1)
    mu = {0: 2.0 / sigma ** 2}
    for d in range(n):
        for node in range(1 << d):
            p = (1 << d) + node - 1
            m = mu[p]
            mu_f[p] = _phi_inv(1 - (1 - float(_phi(m))) ** 2)
            mu_g[p] = 2 * m
            mu[2 * p + 1] = mu_f[p]
            mu[2 * p + 2] = mu_g[p]
    return mu_f, mu_g


def ga_uniform(N: int, sigma: float, v: int = 16) -> UniformQuant:
    """Uniform steps covering mean + 3 std of the GA LLR density at each node."""
    mu_f, mu_g = ga_means(N, sigma)
    span = lambda m: m + 3 * np.sqrt(2 * m)  # noqa: E731
    return UniformQuant(int(N), int(v), span(mu_f) / (v / 2), span(mu_g) / (v / 2))


def ga_lloyd(N: int, sigma: float, v: int = 16) -> LloydQuant:
    """v cells: -inf, v-1 uniform boundaries over +-(mean + 3 std), +inf; cell midpoints."""
    mu_f, mu_g = ga_means(N, sigma)
    bf, bg, rf, rg = [], [], [], []
    for m_all, B, R in ((mu_f, bf, rf), (mu_g, bg, rg)):
        for m in m_all:
            s = m + 3 * np.sqrt(2 * m)
            inner = np.linspace(-s, s, v - 1)
            b = np.concatenate([[-np.inf], inner, [np.inf]])
            r = np.empty(v)
            r[1:-1] = 0.5 * (inner[:-1] + inner[1:])
            r[0] = inner[0] - 0.5 * (inner[1] - inner[0])
            r[-1] = inner[-1] + 0.5 * (inner[1] - inner[0])
            B.append(b)
            R.append(r)
    return pack_lloyd(N, np.array(bf), np.array(bg), np.array(rf), np.array(rg), v)
