#!/usr/bin/env python3
"""Throughput benchmark: decoded frames/s of the N=1024 K=512 SCL-LUT (L=8,
Q=16) decoder (BASELINE.json `metric`, configs[2]), 1..8 MI355X.

A step = one decode launch over one batch of synthetic AWGN frames that are
already resident in HBM.  With --gpus N>1 the driver runs this under
torch.distributed.run; every rank decodes its own disjoint frame range (weak
scaling, no collective on the data path) and the only collective is the RCCL
all-reduce of the error counters {bit errors, block errors, frames}.

Rank 0 prints one JSON line (contract in the task statement), including
`roofline` for the decode kernel (HIP-event timing on the launch stream) and
`cpu_baseline` (the reference decoder compiled from its sources, oracle/_ref,
timed on one host core over a bounded sample of the same workload).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
LDS_PEAK_GBS = 150000.0  # MI355X_MICROARCH.md §LDS: ds_read_b64/b128 aggregate, every CU streaming
LOOKUPS_PER_FRAME = 81920  # L*N*log2(N) LUT lookups at N=1024, L=8
ONCHIP_BYTES_PER_LOOKUP = 4


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--kind", default="SCL-LUT", choices=["SC-LUT", "SCL-LUT", "FastSC-LUT", "FastSCL-LUT"])
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--K", type=int, default=512)
    ap.add_argument("--L", type=int, default=8)
    ap.add_argument("--frames", type=int, default=1 << 18, help="frames per GPU per step")
    ap.add_argument("--ebn0", type=float, default=2.0)
    ap.add_argument("--max-waves", type=int, default=0)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--engine", default="auto", choices=["auto", "fast", "generic"])
    return ap.parse_args()


def synth_frames(N, K, frames, ebn0, seed, msgbits, dev, v=16, delta=0.5):
    """Reference driver channel (mainQuantizedDecoder_LLRDomain.py:132-176), generated
    on the GPU with torch's counter-based RNG: message bits, polar encoding
    (x = u F^{(x)n}, the un-vendored PolarEnc restated), BPSK, AWGN at Eb/N0,
    LLR = 2y/sigma^2 and a uniform 16-level channel quantizer matching the
    synthetic min-sum tables.  Returns device tensors (msg uint8 [F,K], sym int32 [F,N])."""
    import torch

    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    sigma = float(np.sqrt(1 / (2 * (K / N) * 10 ** (ebn0 / 10))))
    msg = torch.randint(0, 2, (frames, K), generator=g, device=dev, dtype=torch.uint8)
    u = torch.zeros((frames, N), dtype=torch.uint8, device=dev)
    u[:, torch.as_tensor(msgbits, device=dev)] = msg
    m = 1
    while m < N:
        w = u.view(frames, N // (2 * m), 2, m)
        w[:, :, 0, :] ^= w[:, :, 1, :]
        m *= 2
    llr = (1.0 - 2.0 * u.float() + sigma * torch.randn((frames, N), generator=g, device=dev)) * (2 / sigma ** 2)
    sym = torch.clamp(torch.round(llr / delta + (v - 1) / 2.0), 0, v - 1).to(torch.int32)
    return msg, sym


def cpu_baseline(args, packed, fm, nt, sym, seconds):
    """Reference decoder (oracle/_ref, compiled from /root/reference sources) on
    one core; falls back to the oracle restatement (kind "port")."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from quantized_decoder_polar_codes_amd import lut as LU

    R = oracle.reference_module()
    N, K, L = args.N, args.K, args.L
    if R is not None:
        fs, gs, vcl = LU.unpack_to_reference(packed)
        fz, mm = fm.astype(int).tolist(), (1 - fm).astype(int).tolist()
        ctor = {"SC-LUT": lambda: R.SCLUTDecoder(N, K, fz, mm, fs, gs, vcl),
                "SCL-LUT": lambda: R.SCLLUTDecoder(N, K, L, fz, mm, fs, gs, vcl),
                "FastSC-LUT": lambda: R.FastSCLUTDecoder(N, K, fz, mm, nt.tolist(), fs, gs, vcl),
                "FastSCL-LUT": lambda: R.FastSCLLUTDecoder(N, K, L, fz, mm, nt.tolist(), fs, gs, vcl)}
        dec = ctor[args.kind]()
        kind = "reference"
        one = lambda s: dec.decode(s)  # noqa: E731
    else:
        kind = "port"
        one = lambda s: oracle.decode_lut(args.kind, packed, K, L, fm, s[None], node_type=nt)[0]  # noqa: E731
    outs = []
    t0 = time.perf_counter()
    i = 0
    while time.perf_counter() - t0 < seconds and i < len(sym):
        outs.append(one(sym[i]))
        i += 1
    dt = time.perf_counter() - t0
    return {"value": i / dt, "unit": "frames/s", "cores": 1, "kind": kind,
            "sample": f"{i} frames of the same workload (first frames of rank 0's batch), one decode() call per "
                      f"frame, single thread, {dt:.1f} s"}, np.stack(outs)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")  # RCCL over xGMI
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    import quantized_decoder_polar_codes_amd as Q
    from quantized_decoder_polar_codes_amd import codes as C
    from quantized_decoder_polar_codes_amd import lut as LU

    N, K, L = args.N, args.K, args.L
    _, mb, fm, mm = C.construct_pw(N, K)
    nt = C.identify_nodes(N, mb).astype(np.int32)
    packed = LU.minsum_uniform_luts(N, v=16, delta=0.5)
    dec = Q.from_packed(args.kind, packed, K, fm, L=L, node_type=nt, device=dev.index, max_waves=args.max_waves,
                        engine=args.engine)
    info = dec.info()
    # rank r owns global frames [r*F, (r+1)*F): seed by rank -> disjoint frame sets
    d_msg, d_sym = synth_frames(N, K, args.frames, args.ebn0, 1234 + rank, mb, dev)
    stream = torch.cuda.current_stream(dev)

    out = None
    for _ in range(args.warmup):
        out = dec.decode_batch(d_sym)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        out = dec.decode_batch(d_sym)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / max(1, args.steps)  # kernel launches on this stream, per step

    # error counters (BER/BLER) -- the only collective: RCCL all-reduce
    err = (out != d_msg)
    cnt = torch.tensor([int(err.sum().item()), int(err.any(1).sum().item()), args.frames], dtype=torch.int64, device=dev)
    tmax = torch.tensor([wall], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(cnt, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    wall = float(tmax.item())
    bit_errs, blk_errs, frames_all = (int(x) for x in cnt.tolist())
    total_frames = args.frames * world * args.steps
    value = total_frames / wall

    if rank == 0:
        frames_per_launch = args.frames
        hbm_bytes = frames_per_launch * (N * 4 + K)  # int32 symbols in, uint8 bits out
        achieved = hbm_bytes / (kern_ms * 1e-3) / 1e9
        onchip = frames_per_launch * LOOKUPS_PER_FRAME * ONCHIP_BYTES_PER_LOOKUP * (L / 8) * (N / 1024) \
            / (kern_ms * 1e-3) / 1e9
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc):
            try:
                rec = json.load(open(pmc))
                key = f"{args.kind}_N{N}_K{K}_L{L}_F{frames_per_launch}"
                traffic = rec.get(key)
            except Exception:
                traffic = None
        res = {
            "metric": "decoded frames/sec (N=1024, SCL-LUT L=8, Q=16) at 1/2/4/8 GPUs; BER match",
            "value": value,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic, generated on the GPU (torch Philox): random messages, polar-encoded, BPSK + AWGN at Eb/N0 below, uniform 16-level channel quantizer, "
                    "synthetic saturating min-sum 16-level LUTs; resident in HBM",
            "config": {"workload": f"{args.kind} N={N} K={K} L={L} Q=16 (5G-NR PW code, no CRC)",
                       "decoder": args.kind, "N": N, "K": K, "L": L, "v": 16, "frames_per_gpu_per_step": args.frames,
                       "ebn0_db": args.ebn0, "parallelism": f"dp{world} (frames sharded, RCCL counter all-reduce)",
                       "engine": {1: "generic", 2: "fast"}[info["engine"]], "lds_bytes_per_wave": info["lds_bytes_per_wave"],
                       "lds_from_depth": info["lds_from_depth"], "waves": min(info["max_waves"],
                       -(-args.frames // info["frames_per_wave"]))},
            "ber": bit_errs / max(1, frames_all * K),
            "bler": blk_errs / max(1, frames_all),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel_ms": kern_ms, "algorithmic_bytes_per_launch": hbm_bytes,
                         "onchip_lds_equiv": {"achieved": onchip, "peak": LDS_PEAK_GBS, "unit": "GB/s",
                                              "frac": onchip / LDS_PEAK_GBS,
                                              "bytes_per_frame": LOOKUPS_PER_FRAME * ONCHIP_BYTES_PER_LOOKUP}},
        }
        if world == 1 and not args.no_cpu_baseline:
            sample = d_sym[:4096].cpu().numpy()
            cb, ref_out = cpu_baseline(args, packed, fm, nt, sample, args.cpu_baseline_seconds)
            res["cpu_baseline"] = cb
            gpu_out = out[: len(ref_out)].cpu().numpy()
            res["parity_sample"] = {"frames": int(len(ref_out)),
                                    "bit_exact_vs_" + cb["kind"]: bool((gpu_out == ref_out).all())}
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
