"""Monte-Carlo BER/BLER harness -- the reference driver's loop, GPU-resident and
sharded across ranks.

Reference semantics (mainQuantizedDecoder_LLRDomain.py:130-203), reproduced
exactly for the frame sequence f = 0, 1, 2, ... of one Eb/N0 point:

    Nbiterrs += errors(f);  Nblkerrs += any_error(f)
    if Nblkerrs > stop:  BER = Nbiterrs / (A * Nblocks);  BLER = Nblkerrs / Nblocks;  stop
    Nblocks += 1
    if Nblocks == MaxBlock:  BER = Nbiterrs / (K * Nblocks);  BLER = Nblkerrs / Nblocks

(the frame that crosses the threshold is counted in the error totals but not in
Nblocks).  Frames are produced by ``qpd_mc_frames`` keyed by GLOBAL frame id, so
the union of frames -- and hence every counter -- is identical for any number
of ranks.  Each step processes ``world * batch`` consecutive frames, rank r
taking the r-th slice; the only collective is an all-reduce of two counters per
step (plus one all-gather of per-frame error counts in the step that crosses
the stop threshold, to locate the exact frame).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib


@dataclass
class PointResult:
    ebn0_db: float
    ber: float
    bler: float
    bit_errors: int
    block_errors: int
    blocks: int
    frames_decoded: int
    stopped_early: bool


def uniform_channel_quantizer(v: int = 16, delta: float = 0.5):
    """Edges/lut of a uniform v-level channel quantizer in the driver's format
    (interval_x with v+1 edges, channel_lut with v entries)."""
    edges = delta * (np.arange(v + 1, dtype=np.float64) - v / 2.0)
    return edges, np.arange(v, dtype=np.int32)


def sigma_for(ebn0_db: float, rate: float) -> float:
    """mainQuantizedDecoder_LLRDomain.py:132-133."""
    return float(np.sqrt(1.0 / (2.0 * rate * 10 ** (ebn0_db / 10.0))))


def point_seed(seed: int, ebn0_db: float) -> int:
    return (int(seed) * 1000003 + int(round(ebn0_db * 1000))) & 0xFFFFFFFFFFFFFFFF


class GpuFrames:
    """Frame source backed by qpd_mc_frames (device tensors)."""

    def __init__(self, decoder, edges, lut, q: int, sigma: float, seed: int):
        import torch

        self.torch = torch
        self.dec = decoder
        self.edges = np.ascontiguousarray(edges, dtype=np.float64)
        self.lut = np.ascontiguousarray(lut, dtype=np.int32)
        self.ch = _lib.QpdMcChannel()
        self.ch.sigma = float(sigma)
        self.ch.q = int(q)
        self.ch.n_edges = len(self.edges)
        self.ch.edges = self.edges.ctypes.data
        self.ch.lut = self.lut.ctypes.data
        self.seed = int(seed)
        self.device = torch.device("cuda", decoder.device if decoder.device >= 0 else torch.cuda.current_device())

    def decode_frames(self, frame0: int, B: int, counts=None):
        """(msg, decoded bits) of frames [frame0, frame0+B): the same bits as
        decode_batch(self(frame0, B)[1]), by qpd_mc_decode (generation feeds the
        decode kernel's pre-pass rows directly, no int32 symbols).  ``counts``:
        a device int64[2] tensor the frames' bit and block errors are added to."""
        torch = self.torch
        msg = torch.empty((B, self.dec.out_bits), dtype=torch.uint8, device=self.device)
        bits = torch.empty((B, self.dec.out_bits), dtype=torch.uint8, device=self.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        cp = ctypes.c_void_p(counts.data_ptr()) if counts is not None else None
        _lib.check(_lib.load().qpd_mc_decode(self.dec._h, ctypes.byref(self.ch), ctypes.c_uint64(self.seed), frame0, B,
                                             ctypes.c_void_p(msg.data_ptr()), ctypes.c_void_p(bits.data_ptr()), cp,
                                             ctypes.c_void_p(stream)))
        return msg, bits

    def __call__(self, frame0: int, B: int):
        torch = self.torch
        msg = torch.empty((B, self.dec.out_bits), dtype=torch.uint8, device=self.device)
        sym = torch.empty((B, self.dec.N), dtype=torch.int32, device=self.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        _lib.check(_lib.load().qpd_mc_frames(self.dec._h, ctypes.byref(self.ch), ctypes.c_uint64(self.seed), frame0, B,
                                             ctypes.c_void_p(msg.data_ptr()), ctypes.c_void_p(sym.data_ptr()),
                                             ctypes.c_void_p(stream)))
        return msg, sym


def _frame_errors(bits, msg):
    """Per-frame bit-error counts as a 1-D int64 tensor/array."""
    try:
        import torch

        if isinstance(bits, torch.Tensor):
            return (bits != msg).sum(dim=1, dtype=torch.int64)
    except Exception:  # pragma: no cover
        pass
    return (np.asarray(bits) != np.asarray(msg)).sum(axis=1).astype(np.int64)


def _step_fn(generate, decode, gen_decode):
    """(msg, bits) of a frame range: one fused call, or generate then decode."""
    if gen_decode is not None:
        return gen_decode

    def step(lo, n):
        msg, sym = generate(lo, n)
        return msg, decode(sym)

    return step


def _run_point_all(step_fn, K, ebn0_db, batch, max_blocks, world, rank, group, count_device, counted=None):
    """run_point without early stop (the driver's MaxBlock branch, :194-196):
    counters accumulate on the device, one all-reduce at the end.
    ``counted(frame0, B, counts)``: a fused call that also adds the frames'
    errors to the device counters (GpuFrames.decode_frames)."""
    import torch
    import torch.distributed as dist

    acc = torch.zeros(2, dtype=torch.int64, device=count_device)
    f0 = 0
    while f0 < max_blocks:
        step = min(world * batch, max_blocks - f0)
        lo = f0 + min(rank * batch, step)
        hi = f0 + min((rank + 1) * batch, step)
        if hi > lo:
            if counted is not None and acc.is_cuda:
                counted(lo, hi - lo, acc)
            else:
                msg, bits = step_fn(lo, hi - lo)
                e = _frame_errors(bits, msg)
                e_t = (e if isinstance(e, torch.Tensor) else torch.from_numpy(e)).to(count_device)
                acc[0] += e_t.sum()
                acc[1] += (e_t > 0).sum()
        f0 += step
    if group is not None:
        dist.all_reduce(acc, group=group)
    bit_errs, blk_errs = (int(x) for x in acc.tolist())
    blocks = max_blocks
    return PointResult(ebn0_db, bit_errs / (K * blocks), blk_errs / blocks, bit_errs, blk_errs, blocks, blocks, False)


def run_point(generate, decode, K: int, ebn0_db: float, batch: int, max_blocks: int, stop_blkerrs: int | None = 1000,
              A: int | None = None, group=None, count_device="cpu", gen_decode=None, shard=None,
              virtual_world: int = 1) -> PointResult:
    """Run one Eb/N0 point.  ``generate(frame0, B) -> (msg, sym)`` and
    ``decode(sym) -> bits`` are this rank's frame source and decoder, or
    ``gen_decode(frame0, B) -> (msg, bits)`` does both in one call
    (GpuFrames.decode_frames); ``group`` is a torch.distributed process group
    (None = single process).  ``stop_blkerrs=None``: no early stop (every
    frame up to max_blocks).

    Without a group, two ways to run the sharding of a ``world``-rank job in
    one process (tests of config C5's 8-rank split on one device):
    ``shard=(rank, world)`` (no early stop only) returns rank ``rank``'s
    counters alone, with ``blocks`` / ``frames_decoded`` its own frame count and
    ``ber`` / ``bler`` over those frames -- the ranks' counters summed are the
    job's, which is what the end-of-point all-reduce computes; ``virtual_world=W`` runs the W
    ranks' slices of every step in lock step, combining them as the per-step
    all-reduce / all-gather would (the stop rule's crossing may then fall in
    any rank's slice)."""
    import torch
    import torch.distributed as dist

    A = K if A is None else A
    world = dist.get_world_size(group) if group is not None else 1
    rank = dist.get_rank(group) if group is not None else 0
    if shard is not None:
        assert group is None and stop_blkerrs is None, "shard=(rank, world): no group, no early stop"
        rank, world = shard
    step_fn = _step_fn(generate, decode, gen_decode)
    if stop_blkerrs is None:
        counted = (lambda lo, n, acc: gen_decode(lo, n, counts=acc)) if gen_decode is not None else None
        res = _run_point_all(step_fn, K, ebn0_db, batch, max_blocks, world, rank, group, count_device, counted)
        if shard is not None:  # this rank's frames only: its counters over its own frame count
            n = sum(max(0, min((rank + 1) * batch, min(world * batch, max_blocks - f0)) -
                       min(rank * batch, min(world * batch, max_blocks - f0)))
                    for f0 in range(0, max_blocks, world * batch))
            res.frames_decoded = res.blocks = n
            res.ber = res.bit_errors / (K * n) if n else 0.0
            res.bler = res.block_errors / n if n else 0.0
        return res
    if virtual_world > 1:
        assert group is None, "virtual_world: no group"
        world = virtual_world
    vranks = list(range(world)) if virtual_world > 1 else [rank]

    def local_step(f0, step, r):
        lo = f0 + min(r * batch, step)
        hi = f0 + min((r + 1) * batch, step)
        if hi > lo:
            msg, bits = step_fn(lo, hi - lo)
            e = _frame_errors(bits, msg)
            e_t = e if isinstance(e, torch.Tensor) else torch.from_numpy(e)
            return e_t.to(count_device)
        return torch.zeros(0, dtype=torch.int64, device=count_device)

    bit_errs = blk_errs = 0
    blocks = 0
    f0 = 0
    while f0 < max_blocks:
        step = min(world * batch, max_blocks - f0)
        e_all = [local_step(f0, step, r) for r in vranks]
        tot = sum(torch.stack([e.sum(), (e > 0).sum()]).to(torch.int64) for e in e_all)
        if group is not None:
            dist.all_reduce(tot, group=group)
        step_bits, step_blks = (int(x) for x in tot.tolist())
        if blk_errs + step_blks > stop_blkerrs:
            # locate the frame that crosses the threshold: gather per-frame counts in global order
            pads = []
            for e_t in e_all:
                pad = torch.zeros(batch, dtype=torch.int64, device=count_device)
                pad[: e_t.numel()] = e_t
                pads.append(pad)
            if group is not None:
                parts = [torch.zeros_like(pads[0]) for _ in range(world)]
                dist.all_gather(parts, pads[0], group=group)
            else:
                parts = pads
            per = np.concatenate([parts[r].cpu().numpy()[: max(0, min((r + 1) * batch, step) - min(r * batch, step))]
                                  for r in range(world)])
            for i, ef in enumerate(per):
                bit_errs += int(ef)
                blk_errs += int(ef > 0)
                if blk_errs > stop_blkerrs:
                    blocks = f0 + i
                    return PointResult(ebn0_db, bit_errs / (A * blocks) if blocks else float("inf"),
                                       blk_errs / blocks if blocks else float("inf"), bit_errs, blk_errs, blocks,
                                       f0 + step, True)
            raise AssertionError("threshold crossing not found")  # pragma: no cover
        bit_errs += step_bits
        blk_errs += step_blks
        f0 += step
    blocks = max_blocks
    return PointResult(ebn0_db, bit_errs / (K * blocks), blk_errs / blocks, bit_errs, blk_errs, blocks, blocks, False)


def simulate(decoder, msgbits_count: int, ebn0_list, *, seed: int = 2024, batch: int = 1 << 16,
             max_blocks: int = 10 ** 5, stop_blkerrs: int = 1000, edges=None, lut=None, q: int = 16,
             group=None) -> list:
    """BER/BLER sweep on the GPU with the decoder's own code (GPU frames,
    GPU decode, counters all-reduced over ``group`` with RCCL)."""
    import torch

    if edges is None:
        edges, lut = uniform_channel_quantizer(q)
    rate = msgbits_count / decoder.N
    out = []
    for eb in ebn0_list:
        src = GpuFrames(decoder, edges, lut, q, sigma_for(eb, rate), point_seed(seed, eb))
        # CRC-aided decoders output A bits: errors are counted over A, and the
        # driver's BER denominators are A (early stop) / K (MaxBlock), :185,196
        res = run_point(src, decoder.decode_batch, decoder.K, eb, batch, max_blocks, stop_blkerrs, A=decoder.out_bits,
                        group=group, count_device=src.device, gen_decode=src.decode_frames)
        torch.cuda.synchronize()
        out.append(res)
    return out
