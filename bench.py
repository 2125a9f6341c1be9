#!/usr/bin/env python3
"""Throughput benchmark: decoded frames/s of the N=1024 K=512 SCL-LUT (L=8,
Q=16) decoder (BASELINE.json `metric`, configs[2]), 1..8 MI355X.

A step = one decode launch over one batch of synthetic AWGN frames that are
already resident in HBM.  The workload is the reference driver's
(mainQuantizedDecoder_LLRDomain.py:130-176): frames from the GPU Monte-Carlo
generator (qpd_mc_frames: Philox4x32-10 keyed by global frame id, polar
encoding, BPSK + AWGN at Eb/N0, LLR), the MinDistortion channel quantizer
designed at that Eb/N0, and MinDistortion decoder tables designed at 3 dB
(lutgen.py, the reference generator's algorithm).  With --gpus N>1 the driver runs this under
torch.distributed.run; every rank decodes its own disjoint frame range (weak
scaling, no collective on the data path) and the only collective is the RCCL
all-reduce of the error counters {bit errors, block errors, frames}.

Rank 0 prints one JSON line (contract in the task statement), including
`roofline` for the decode kernel (HIP-event timing on the launch stream) and
`cpu_baseline` (the reference decoder compiled from its sources, oracle/_ref,
one worker process per host core of this GPU's CPU share, over a bounded
sample of the same frames).
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
    ap.add_argument("--kind", default="SCL-LUT", choices=["SC-LUT", "SCL-LUT", "FastSC-LUT", "FastSCL-LUT", "CA-SCL-LUT",
                                                          "CA-FastSCL-LUT"])
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--K", type=int, default=512)
    ap.add_argument("--L", type=int, default=8)
    ap.add_argument("--frames", type=int, default=1 << 18, help="frames per GPU per step")
    ap.add_argument("--ebn0", type=float, default=2.0)
    ap.add_argument("--max-waves", type=int, default=0)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--engine", default="auto", choices=["auto", "fast", "generic"])
    ap.add_argument("--luts", default="mindistortion", choices=["mindistortion", "minsum"],
                    help="decoder tables: MinDistortion design (lutgen.py) or synthetic saturating min-sum")
    ap.add_argument("--design-snr", type=float, default=3.0, help="LUT design SNR (dB)")
    ap.add_argument("--cpu-workers", type=int, default=0, help="0 = this GPU's CPU share (OMP_NUM_THREADS, <= 16)")
    return ap.parse_args()


def workload(N, K, L, kind, frames, ebn0, luts="mindistortion", design_snr=3.0, frame0=0, device=None, **dec_kw):
    """The benchmark workload: (decoder, packed tables, frozen mask, node types,
    device msg uint8 [F, K], device symbols int32 [F, N]) -- see the module doc."""
    import quantized_decoder_polar_codes_amd as Q
    from quantized_decoder_polar_codes_amd import codes as C
    from quantized_decoder_polar_codes_amd import lut as LU
    from quantized_decoder_polar_codes_amd import lutgen as LG
    from quantized_decoder_polar_codes_amd import montecarlo as MC

    _, mb, fm, mm = C.construct_pw(N, K)
    nt = C.identify_nodes(N, mb).astype(np.int32)
    sigma = MC.sigma_for(ebn0, K / N)  # mainQuantizedDecoder_LLRDomain.py:132-133
    if luts == "mindistortion":
        packed = LG.design(N, 16, design_snr).packed()
        _, _, edges, clut = LG.channel_quantizer(sigma, 128, 16)  # the driver's per-Eb/N0 channel quantizer
    else:
        packed = LU.minsum_uniform_luts(N, v=16, delta=0.5)
        edges, clut = MC.uniform_channel_quantizer(16, 0.5)
    if kind.startswith("CA-"):  # CRC-aided: A = K - 24 message bits + CRC-24 (the drivers' K = A + crc_n)
        dec_kw.setdefault("A", K - 24)
    dec = Q.from_packed(kind, packed, K, fm, L=L, node_type=nt, device=device, **dec_kw)
    src = MC.GpuFrames(dec, edges, clut, 16, sigma, seed=1234)  # Philox keyed by global frame id
    msg, sym = src(frame0, frames)
    return dec, packed, fm, nt, msg, sym


_WORKER = r"""
import sys, time, json
import numpy as np
sys.path.insert(0, ROOT); sys.path.insert(0, ROOT + "/oracle")
import oracle
from quantized_decoder_polar_codes_amd import lut as LU
z = np.load(PATH, allow_pickle=False)
R = oracle.reference_module()
N, K, L, kind, A = int(z["N"]), int(z["K"]), int(z["L"]), str(z["kind"]), int(z["A"])
packed = LU.PackedLUT(N=N, v=int(z["v"]), lut_f=z["lut_f"], f_base=z["f_base"], f_step=0, lut_g=z["lut_g"],
                      g_base=z["g_base"], g_step=0, vcl=np.ascontiguousarray(z["vcl"]))
fm, nt, sym = z["frozen"], z["node_type"], z["sym"]
if R is not None:
    fs, gs, vcl = LU.unpack_to_reference(packed)
    fz, mm = fm.astype(int).tolist(), (1 - fm).astype(int).tolist()
    dec = {"SC-LUT": lambda: R.SCLUTDecoder(N, K, fz, mm, fs, gs, vcl),
           "SCL-LUT": lambda: R.SCLLUTDecoder(N, K, L, fz, mm, fs, gs, vcl),
           "FastSC-LUT": lambda: R.FastSCLUTDecoder(N, K, fz, mm, nt.tolist(), fs, gs, vcl),
           "FastSCL-LUT": lambda: R.FastSCLLUTDecoder(N, K, L, fz, mm, nt.tolist(), fs, gs, vcl),
           "CA-SCL-LUT": lambda: R.CASCLLUTDecoder(N, K, A, L, fz, mm, 24, list(oracle.CRC24_LOC), fs, gs, vcl),
           "CA-FastSCL-LUT": lambda: R.CAFastSCLLUTDecoder(N, K, A, L, fz, mm, nt.tolist(), fs, gs, vcl)}[kind]()
    one = dec.decode
else:
    one = (lambda s: oracle.decode_lut_ca(kind, packed, K, A, L, fm, s[None], node_type=nt)[0]) if kind.startswith("CA-") \
        else (lambda s: oracle.decode_lut(kind, packed, K, L, fm, s[None], node_type=nt)[0])
outs = []
t0 = time.perf_counter()
while time.perf_counter() - t0 < SECONDS and len(outs) < len(sym):
    outs.append(one(sym[len(outs)]))
dt = time.perf_counter() - t0
np.save(PATH + ".out.npy", np.stack(outs).astype(np.uint8))
print(json.dumps({"frames": len(outs), "seconds": dt, "kind": "reference" if R is not None else "port"}))
"""


def cpu_baseline(args, packed, fm, nt, sym, seconds, workers, A):
    """The reference decoder (oracle/_ref, compiled from /root/reference sources;
    the oracle restatement, kind "port", if that build is absent), one worker
    process per core, each decoding its own slice of the sample one frame per
    decode() call for `seconds`.  Workers are plain child processes (no GPU)."""
    import subprocess
    import tempfile

    per = len(sym) // workers
    tmp = tempfile.mkdtemp(prefix="qpd_cpu_")
    procs = []
    for w in range(workers):
        path = os.path.join(tmp, f"w{w}.npz")
        np.savez(path, N=args.N, K=args.K, A=A, L=args.L, kind=args.kind, v=packed.v, lut_f=packed.lut_f,
                 f_base=packed.f_base, lut_g=packed.lut_g, g_base=packed.g_base, vcl=packed.vcl, frozen=fm,
                 node_type=nt, sym=sym[w * per:(w + 1) * per])
        code = _WORKER.replace("ROOT", repr(ROOT)).replace("PATH", repr(path)).replace("SECONDS", repr(seconds))
        procs.append((subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, text=True), path))
    total, walls, outs, kind = 0, [], [], "port"
    for w, (p, path) in enumerate(procs):
        o, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"cpu baseline worker {w} failed")
        r = json.loads(o.strip().splitlines()[-1])
        total += r["frames"]
        walls.append(r["seconds"])
        kind = r["kind"]
        outs.append((w * per, np.load(path + ".out.npy")))
    import shutil

    shutil.rmtree(tmp, ignore_errors=True)
    wall = max(walls)
    return {"value": total / wall, "unit": "frames/s", "cores": workers, "kind": kind,
            "sample": f"{total} frames of the same workload (rank 0's first frames), {workers} worker processes x "
                      f"one decode() call per frame, {wall:.1f} s"}, outs


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

    N, K, L = args.N, args.K, args.L
    # rank r owns global frames [r*F, (r+1)*F) of one Philox stream
    dec, packed, fm, nt, d_msg, d_sym = workload(N, K, L, args.kind, args.frames, args.ebn0, args.luts, args.design_snr,
                                                 frame0=rank * args.frames, device=dev.index,
                                                 max_waves=args.max_waves, engine=args.engine)
    info = dec.info()
    torch.cuda.synchronize()
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
            "data": ("synthetic, generated on the GPU by qpd_mc_frames (Philox4x32-10 keyed by global frame id): random "
                     "messages, polar-encoded, BPSK + AWGN at Eb/N0 below, the driver's MinDistortion channel quantizer "
                     f"(128 -> 16 levels); decoder tables: {args.luts}"
                     + (f" designed at {args.design_snr:g} dB by lutgen.py" if args.luts == "mindistortion" else "")
                     + "; resident in HBM"),
            "config": {"workload": f"{args.kind} N={N} K={K} L={L} Q=16 (5G-NR PW code, no CRC)",
                       "decoder": args.kind, "N": N, "K": K, "L": L, "v": 16, "frames_per_gpu_per_step": args.frames,
                       "ebn0_db": args.ebn0, "luts": args.luts, "parallelism": f"dp{world} (frames sharded, RCCL counter all-reduce)",
                       "engine": {1: "generic", 2: "fast"}[info["engine"]], "lds_bytes_per_wave": info["lds_bytes_per_wave"],
                       "lds_from_depth": info["lds_from_depth"], "waves": min(info["max_waves"],
                       -(-args.frames // info["frames_per_wave"]))},
            "ber": bit_errs / max(1, frames_all * dec.out_bits),
            "bler": blk_errs / max(1, frames_all),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel_ms": kern_ms, "algorithmic_bytes_per_launch": hbm_bytes,
                         "kernels": "one decode call = root_pre_kernel + lut_fast_kernel on the bench stream "
                                    "(HIP events bracket both; traffic sums both)" if info["engine"] == 2 else
                                    "generic_decode_kernel",
                         "onchip_lds_equiv": {"achieved": onchip, "peak": LDS_PEAK_GBS, "unit": "GB/s",
                                              "frac": onchip / LDS_PEAK_GBS,
                                              "bytes_per_frame": LOOKUPS_PER_FRAME * ONCHIP_BYTES_PER_LOOKUP}},
        }
        if world == 1 and not args.no_cpu_baseline:
            workers = args.cpu_workers or min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)))
            sample = d_sym[: 1 << 15].cpu().numpy()
            cb, parts = cpu_baseline(args, packed, fm, nt, sample, args.cpu_baseline_seconds, max(1, workers),
                                     dec.out_bits)
            res["cpu_baseline"] = cb
            gpu_out = out.cpu().numpy()
            ok = all(np.array_equal(gpu_out[o:o + len(r)], r) for o, r in parts)
            res["parity_sample"] = {"frames": int(sum(len(r) for _, r in parts)), "bit_exact_vs_" + cb["kind"]: bool(ok)}
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
