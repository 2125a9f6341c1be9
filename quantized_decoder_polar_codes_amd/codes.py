"""Host-side code utilities that produce the decoder's inputs.

These are restatements (numpy-2 safe) of the reference's host helpers:

* ``construct_pw``     -- PolarCodeConstructor.PW, PolarCodesUtils/CodeConstruction.py:65-84
* ``identify_nodes``   -- NodeIdentifier.run, PolarCodesUtils/IdentifyNodes.py:13-150
* ``polar_encode``     -- the un-vendored PolarBDEnc ``PolarEnc.encode`` (natural-order
  x = u F^{(x)n}), the same butterfly the reference decoders use to re-encode
  (FastSCLUT.cpp:186-198)
* ``channel_llr_density_table`` -- utils.py:30-45 (channel quantizer design input)

They run once per code (or per Eb/N0 point) on the host; none of them is on
the decode hot path.
"""
from __future__ import annotations

import os
from bisect import bisect_left

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))


def reliability_sequence() -> np.ndarray:
    """5G-NR polar reliability sequence (3GPP TS 38.212 Table 5.3.1.2-1), Nmax=1024,
    least reliable first -- the data of the reference's ``reliable sequence.txt``."""
    with open(os.path.join(_HERE, "reliability_nr.txt")) as fh:
        return np.array([int(t) for t in fh.read().split()], dtype=np.int64)


def construct_pw(N: int, K: int):
    """5G-NR construction (CodeConstruction.py:71-84): the N-K least reliable
    sub-channels (< N) are frozen.  Returns (frozenbits, msgbits, frozen_mask,
    message_mask) with int64 masks, 1 = frozen / 1 = message."""
    if N > 1024 or N < 2 or N & (N - 1):
        raise ValueError("construct_pw supports power-of-two N in [2, 1024]")
    if not 0 <= K <= N:
        raise ValueError("K must be in [0, N]")
    q = reliability_sequence()
    q = q[q < N]
    frozenbits = np.sort(q[: N - K])
    frozen_mask = np.zeros(N, dtype=np.int64)
    frozen_mask[frozenbits] = 1
    msgbits = np.flatnonzero(frozen_mask == 0)
    message_mask = 1 - frozen_mask
    return frozenbits, msgbits, frozen_mask, message_mask


# Node type labels, IdentifyNodes.py:19-28.
R0, R1, REP, SPC = 0, 1, 2, 3


def identify_nodes(N: int, msgbits, use_new_node: bool = False) -> np.ndarray:
    """Label decoding-tree nodes (IdentifyNodes.py:13-150).

    Returns a float64 array of length 2N-1 indexed by node_posi = 2^depth+node-1
    (the drivers cast it with ``.astype(np.int32)``).  A node is labelled at its
    first visit by the pattern of information bits under it; descendants of a
    labelled node stay -1 because the identifier never descends into it.  Leaves
    reached by the traversal are labelled 0 (frozen) / 1 (message).
    """
    n = int(np.log2(N))
    info = np.zeros(N, dtype=np.int64)
    info[np.asarray(msgbits, dtype=np.int64)] = 1
    node_type = -np.ones(2 * N - 1)

    def classify(seg):
        t = len(seg)
        s = int(seg.sum())
        if s == 0:
            return R0
        if s == t:
            return R1
        if s == 1 and seg[-1] == 1:
            return REP
        if s == t - 1 and seg[0] == 0:
            return SPC
        if use_new_node:
            if s == 2 and seg[-1] == 1 and seg[-2] == 1 and t >= 4:
                return 4
            if s == 3 and seg[-1] == 1 and seg[-2] == 1 and seg[-3] == 1 and t >= 4:
                return 5
            if s == t - 2 and seg[0] == 0 and seg[1] == 0 and t >= 4:
                return 6
            if s == t - 3 and seg[0] == 0 and seg[1] == 0 and seg[2] == 0 and t >= 4:
                return 7
            if s == 4 and seg[-1] == 1 and seg[-2] == 1 and seg[-3] == 1 and seg[-5] == 1 and t >= 8:
                return 8
        return None

    def visit(depth, node):
        posi = (1 << depth) + node - 1
        if depth == n:
            node_type[posi] = 1 if info[node] else 0
            return
        temp = N >> depth
        t = classify(info[temp * node: temp * (node + 1)])
        if t is not None:
            node_type[posi] = t
            return
        visit(depth + 1, 2 * node)
        visit(depth + 1, 2 * node + 1)

    visit(0, 0)
    return node_type


def polar_transform(u: np.ndarray) -> np.ndarray:
    """x = u F^{(x)n} in natural order over the last axis (bitwise XOR butterflies)."""
    x = np.array(u, dtype=np.uint8, copy=True)
    N = x.shape[-1]
    m = 1
    while m < N:
        v = x.reshape(x.shape[:-1] + (N // (2 * m), 2, m))
        v[..., 0, :] ^= v[..., 1, :]
        m *= 2
    return x


def polar_encode(msg: np.ndarray, msgbits, N: int) -> np.ndarray:
    """Restated PolarEnc.encode: u[msgbits] = msg, frozen = 0, x = u F^{(x)n}.
    ``msg`` may be [K] or [B, K]."""
    msg = np.asarray(msg, dtype=np.uint8)
    u = np.zeros(msg.shape[:-1] + (N,), dtype=np.uint8)
    u[..., np.asarray(msgbits)] = msg
    return polar_transform(u)


def channel_llr_density_table(M, low, high, mu1, mu2, sigma):
    """utils.py:30-45 -- binned two-Gaussian LLR density used to design the
    channel quantizer.  Returns (pyx, x_discrete, quanta)."""
    delta = 0.0001
    x_continuous = np.arange(low, high + delta, delta)
    pyx_continuous = 0.5 * (
        1 / np.sqrt(2 * np.pi * sigma ** 2) * np.exp(-((x_continuous - mu1) ** 2) / (2 * sigma ** 2))
        + 1 / np.sqrt(2 * np.pi * sigma ** 2) * np.exp(-((x_continuous - mu2) ** 2) / (2 * sigma ** 2))
    )
    x_discrete = np.linspace(low, high, M + 1)
    quanta = np.zeros(M)
    pyx = np.zeros(M)
    for i in range(M):
        index = np.bitwise_and(x_continuous >= x_discrete[i], x_continuous <= x_discrete[i + 1])
        density = pyx_continuous[index]
        pyx[i] = np.sum(density) * delta
        quanta[i] = np.sum(x_continuous[index] * density) / np.sum(density)
    return pyx, x_discrete, quanta


def quantize_channel(llr: np.ndarray, interval_x: np.ndarray, channel_lut: np.ndarray, q_channel: int) -> np.ndarray:
    """Channel LLR -> decoder input symbols, mainQuantizedDecoder_LLRDomain.py:167-176:
    saturate at the outer edges, otherwise ``channel_lut[bisect_left(edges[:-1], llr) - 1]``."""
    llr = np.asarray(llr, dtype=np.float64)
    edges = np.asarray(interval_x, dtype=np.float64)
    lut = np.asarray(channel_lut).reshape(-1)
    idx = np.searchsorted(edges[:-1], llr, side="left")  # == bisect_left
    out = lut[np.clip(idx - 1, 0, len(lut) - 1)].astype(np.int32)
    out = np.where(llr <= edges[0], 0, out)
    out = np.where(llr >= edges[-1], q_channel - 1, out)
    return out.astype(np.int32)


def quantize_channel_scalar(llr_row, interval_x, channel_lut, q_channel):
    """Per-element loop form of :func:`quantize_channel` (the driver's literal
    loop), kept for tests of the vectorised version."""
    out = np.zeros(len(llr_row), dtype=np.int32)
    for i, x in enumerate(llr_row):
        if x <= interval_x[0]:
            out[i] = 0
        elif x >= interval_x[-1]:
            out[i] = q_channel - 1
        else:
            out[i] = channel_lut[bisect_left(list(interval_x[:-1]), x) - 1]
    return out
