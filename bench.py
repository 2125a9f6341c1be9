#!/usr/bin/env python3
"""Throughput benchmark: decoded frames/s of the N=1024 K=512 SCL-LUT (L=8,
Q=16) decoder (BASELINE.json `metric`, configs[2]), 1..8 MI355X.

A step = one decode launch over one batch of synthetic AWGN frames that are
already resident in HBM.  The workload is the reference driver's
(mainQuantizedDecoder_LLRDomain.py:130-176): frames from the GPU Monte-Carlo
generator (qpd_mc_frames: Philox4x32-10 keyed by global frame id, polar
encoding, BPSK + AWGN at Eb/N0, LLR), the MinDistortion channel quantizer
designed at that Eb/N0, and MinDistortion decoder tables designed at 3 dB
(lutgen.py, the reference generator's algorithm).

Multi-GPU: one process per GPU.  `--gpus N` with N > 1 and
no WORLD_SIZE in the environment re-launches this script under
`torch.distributed.run` (a child process; nothing here has touched the GPU
yet), so `python bench.py --gpus 8` and the driver's own torchrun launch run
the same per-rank body (`run_rank`): rank r decodes global frames
[r*F, (r+1)*F) of one Philox stream (weak scaling, no collective on the data
path) and the only collectives are the RCCL all-reduces of the error counters
{bit errors, block errors, frames} and of the timed wall (max over ranks).

`--mc-frames F` runs BASELINE config 5 instead: a Monte-Carlo point of F
frames (default no early stop, the driver's MaxBlock branch; `--mc-stop 1000`
= its `Nblkerrs > 1000` rule, mainQuantizedDecoder_LLRDomain.py:130-203)
sharded over the ranks by global frame id (montecarlo.run_point), and reports
BER/BLER plus the end-to-end rate (generate + decode + count).

Rank 0 prints one JSON line (contract in the task statement), including
`roofline` for the decode kernel (HIP events around each of its launches on
the launch stream; on-chip bytes against the guide's aggregate LDS rate) and
`cpu_baseline` + `parity_sample` (the reference decoder compiled from its sources, oracle/_ref,
one worker process per host core of this GPU's CPU share, over a bounded
sample of the same frames).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
GUIDE_LDS_B32_GBS = 75000.0  # MI355X_MICROARCH.md §LDS: aggregate ds_read_b32, every CU streaming
GUIDE_LDS_B64_GBS = 150000.0  # ... ds_read_b64 / b128
ONCHIP_BYTES_PER_LOOKUP = 4  # 2 operand symbols + 1 table byte + 1 result byte
METRIC = "decoded frames/sec (N=1024, SCL-LUT L=8, Q=16) at 1/2/4/8 GPUs; BER match"
KINDS = ["SC-LUT", "SCL-LUT", "FastSC-LUT", "FastSCL-LUT", "CA-SCL-LUT", "CA-FastSCL-LUT"]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--kind", default="SCL-LUT", choices=KINDS)
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--K", type=int, default=512)
    ap.add_argument("--L", type=int, default=8)
    ap.add_argument("--frames", type=int, default=1 << 23,
                    help="frames per GPU per step (one decode launch: 2^23 x 4 KB int32 symbols = 32 GB resident)")
    ap.add_argument("--ebn0", type=float, default=2.0)
    ap.add_argument("--max-waves", type=int, default=0)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the generate+decode+count rate")
    ap.add_argument("--engine", default="auto", choices=["auto", "fast", "generic"])
    ap.add_argument("--luts", default="mindistortion", choices=["mindistortion", "minsum"],
                    help="decoder tables: MinDistortion design (lutgen.py) or synthetic saturating min-sum")
    ap.add_argument("--design-snr", type=float, default=3.0, help="LUT design SNR (dB)")
    ap.add_argument("--cpu-workers", type=int, default=0, help="0 = this GPU's CPU share (OMP_NUM_THREADS, <= 16)")
    ap.add_argument("--mc-frames", type=float, default=0,
                    help="Monte-Carlo mode (BASELINE config 5): frames of one Eb/N0 point over all ranks, e.g. 1e8")
    ap.add_argument("--mc-stop", type=int, default=0,
                    help="Monte-Carlo early stop: Nblkerrs > this (the driver uses 1000); 0 = run all frames")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# launch
# ---------------------------------------------------------------------------

def launch_cmd(args, argv, port):
    """The torch.distributed.run command that runs this script on args.gpus ranks."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def self_launch(args, argv) -> int:
    """Run the N-rank job as a child process (this process never touches the GPU)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this pool
    return subprocess.call(launch_cmd(args, argv, port), env=env)


# ---------------------------------------------------------------------------
# workload
# ---------------------------------------------------------------------------

class Workload:
    """This rank's decoder and frames: dec (decode_batch/info/out_bits), the
    frame source src(frame0, B) -> (msg, sym), packed tables, frozen mask and
    node types (for the CPU baseline), and this rank's resident batch."""

    def __init__(self, dec, src, packed, fm, nt, msg, sym, frame0):
        self.dec, self.src, self.packed, self.fm, self.nt = dec, src, packed, fm, nt
        self.msg, self.sym, self.frame0 = msg, sym, frame0


def workload(N, K, L, kind, frames, ebn0, luts="mindistortion", design_snr=3.0, frame0=0, device=None, **dec_kw):
    """The benchmark workload (see the module doc)."""
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
    msg, sym = src(frame0, frames) if frames else (None, None)
    return Workload(dec, src, packed, fm, nt, msg, sym, frame0)


# ---------------------------------------------------------------------------
# the per-rank body
# ---------------------------------------------------------------------------

class Ctx:
    """Where this rank runs: device, process group (None = single process) and
    the device synchronisation (a no-op on CPU, for the gloo tests)."""

    def __init__(self, rank, world, device, group=None):
        import torch

        self.rank, self.world, self.device, self.group = rank, world, device, group
        self._cuda = device.type == "cuda"
        self._torch = torch

    def sync(self):
        if self._cuda:
            self._torch.cuda.synchronize(self.device)

    def barrier(self):
        self.sync()
        if self.group is not None:
            import torch.distributed as dist

            dist.barrier(group=self.group)
        self.sync()

    def allreduce(self, t, op):
        if self.group is not None:
            import torch.distributed as dist

            if dist.get_backend(self.group) == "gloo" and t.is_cuda:  # rehearsal runs: gloo reduces host tensors
                h = t.cpu()
                dist.all_reduce(h, op=op, group=self.group)
                t.copy_(h)
            else:
                dist.all_reduce(t, op=op, group=self.group)
        return t


def timed_steps(ctx, fn, steps, warmup):
    """W untimed calls of fn, then exactly `steps` calls bracketed by a barrier
    and a device sync on both sides; returns (last result, wall seconds)."""
    out = None
    for _ in range(warmup):
        out = fn()
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = fn()
    ctx.barrier()
    return out, time.perf_counter() - t0


def _has_prof(dec):
    return hasattr(dec, "profile") and hasattr(dec, "kernel_times")


def run_rank(args, ctx, wl):
    """Decode throughput on this rank; returns the result dict on rank 0 (None
    elsewhere).  Counters and the wall are all-reduced over ctx.group."""
    import torch
    import torch.distributed as dist

    dec = wl.dec
    prof = _has_prof(dec) and ctx._cuda
    if prof:
        dec.profile(True)
    out, wall = timed_steps(ctx, lambda: dec.decode_batch(wl.sym), args.steps, args.warmup)
    kt = dec.kernel_times() if prof else {}
    if prof:
        dec.profile(False)

    # error counters (BER/BLER) -- the only collectives: RCCL all-reduces
    err = (out != wl.msg)
    cnt = torch.tensor([int(err.sum().item()), int(err.any(1).sum().item()), int(wl.sym.shape[0])],
                       dtype=torch.int64, device=ctx.device)
    tmax = torch.tensor([wall], dtype=torch.float64, device=ctx.device)
    ctx.allreduce(cnt, dist.ReduceOp.SUM)
    ctx.allreduce(tmax, dist.ReduceOp.MAX)
    wall = float(tmax.item())
    bit_errs, blk_errs, frames_all = (int(x) for x in cnt.tolist())
    if ctx.rank != 0:
        return None
    frames = int(wl.sym.shape[0])
    res = {
        "metric": METRIC,
        "value": frames_all * args.steps / wall,
        "unit": "frames/s",
        "n_gpus": ctx.world,
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
        "config": {"workload": f"{args.kind} N={args.N} K={args.K}{(' L=' + str(args.L)) if 'SCL' in args.kind else ''} Q=16 (5G-NR PW code, no CRC)",
                   "decoder": args.kind, "N": args.N, "K": args.K, "L": args.L, "v": 16,
                   "frames_per_gpu_per_step": frames, "ebn0_db": args.ebn0, "luts": args.luts,
                   "parallelism": f"dp{ctx.world} (frames sharded by global frame id, RCCL counter all-reduce)"},
        "ber": bit_errs / max(1, frames_all * dec.out_bits),
        "bler": blk_errs / max(1, frames_all),
        "frames_counted": frames_all,
    }
    if hasattr(dec, "info"):
        info = dec.info()
        res["config"].update({"engine": {1: "generic", 2: "fast"}[info["engine"]],
                              "lds_bytes_per_wave": info["lds_bytes_per_wave"],
                              "lds_from_depth": info["lds_from_depth"],
                              "ops": info["num_ops"], "prefix_ops": info.get("prefix_ops", 0),
                              "waves": min(info["max_waves"], -(-frames // info["frames_per_wave"]))})
    if kt:
        res["roofline"] = roofline(args, dec, kt, frames, args.steps + args.warmup)
    return res


def _counters_key(args, frames):
    return f"{args.kind}_N{args.N}_K{args.K}_L{args.L}_F{frames}"


def _counters(args, frames):
    """profiles/counters.json record of this configuration (tools/counters.py)."""
    path = os.path.join(ROOT, "profiles", "counters.json")
    try:
        return json.load(open(path)).get(_counters_key(args, frames))
    except Exception:
        return None


VALU_ISSUE_CYCLES = 2  # MI355X_MICROARCH.md §Wave: a wave64 VALU instruction issues over 2 cycles
SIMDS = 1024           # 256 CUs x 4 SIMDs
XCDS = 8


def valu_ceiling(kc):
    """VALU issue share of the decode kernel from its PMC record: the wave64 VALU
    instructions per frame x 2 issue cycles / the SIMD-cycles per frame (1024
    SIMDs x the kernel's cycles: GRBM_GUI_ACTIVE counts every XCD's, so / 8).
    About 0.5 on the list kernels: their nearest ceiling (the LDS fraction is
    about 0.23), DESIGN.md §5."""
    pf = (kc or {}).get("per_frame", {})
    if not pf.get("SQ_INSTS_VALU") or not pf.get("GRBM_GUI_ACTIVE"):
        return None
    simd_cycles = SIMDS * pf["GRBM_GUI_ACTIVE"] / XCDS
    return {"frac": pf["SQ_INSTS_VALU"] * VALU_ISSUE_CYCLES / simd_cycles,
            "insts_per_frame": pf["SQ_INSTS_VALU"], "issue_cycles_per_inst": VALU_ISSUE_CYCLES,
            "simd_cycles_per_frame": simd_cycles,
            "note": "VALU issue share (SQ_INSTS_VALU x 2 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)), the kernel's "
                    "nearest ceiling; from the PMC record named in counters_record"}


def roofline(args, dec, kt, frames, calls):
    """Roofline of the dominant kernel (lut_fast_kernel; generic_decode_kernel
    on the generic engine).  achieved = SURVEY.md §8(d)'s algorithmic on-chip
    bytes -- the f/g table lookups the reference's traversal of this code makes
    (qpd_info.lookups_per_path: N log2 N per path for SC/SCL, fewer where the Fast
    decoders' special nodes skip subtrees) x L paths x 4 B per lookup -- x frames
    per launch (a call of `frames` frames is one launch per pre-pass chunk) / the
    kernel's average launch duration from the HIP events on its stream.  peak =
    the guide's aggregate LDS read rate (MI355X_MICROARCH.md §LDS: ds_read_b32,
    every CU streaming, 75 TB/s); the ds_bpermute rate probed on this GPU (the
    instruction the lookups use) is reported beside it.  `hbm` keeps the
    contract's HBM view of a whole decode call (pre-pass + decode)."""
    import ctypes

    from quantized_decoder_polar_codes_amd import _lib

    dec_ms, n_dec = kt["decode"]
    pre_ms, n_pre = kt["pre"]
    pfx_ms, n_pfx = kt.get("pfx", (0.0, 0))
    # the decode of a launch's frames = lut_prefix_kernel (frozen prefix, list kinds) + lut_fast_kernel
    k_ms = (dec_ms + pfx_ms) / max(1, n_dec)
    call_ms = (dec_ms + pre_ms + pfx_ms) / max(1, calls)
    per_launch = frames * calls / max(1, n_dec)  # frames per decode launch
    info = dec.info()
    paths = args.L if "SCL" in args.kind else 1
    lookups = paths * int(info["lookups_per_path"])
    onchip_per_frame = lookups * ONCHIP_BYTES_PER_LOOKUP
    peaks = {}
    for name, op in (("ds_bpermute_b32", _lib.QPD_PROBE_BPERMUTE), ("ds_read_b32", _lib.QPD_PROBE_READ_B32),
                     ("ds_read_b64", _lib.QPD_PROBE_READ_B64)):
        g = ctypes.c_double()
        _lib.check(_lib.load().qpd_probe_lds(dec.device, op, ctypes.byref(g)))
        peaks[name] = g.value
    peak = GUIDE_LDS_B32_GBS
    achieved = onchip_per_frame * per_launch / (k_ms * 1e-3) / 1e9
    hbm_bytes = frames * (args.N * 4 + dec.out_bits)  # int32 symbols in, uint8 bits out
    rec = _counters(args, frames)
    rec_id = _counters_key(args, frames)
    kname = "lut_fast_kernel" if info["engine"] == 2 else "generic_decode_kernel"
    kc = (rec or {}).get("kernels", {}).get(kname, {})
    out = {"bound": "lds", "achieved": achieved, "peak": peak, "unit": "GB/s", "frac": achieved / peak,
           "peak_source": "MI355X_MICROARCH.md §LDS: aggregate ds_read_b32 with every CU streaming (75 TB/s)",
           "traffic": kc.get("traffic"), "kernel": kname, "kernel_ms": dec_ms / max(1, n_dec), "launches": n_dec,
           # frozen-prefix stages (lut_prefix_kernel): their summed time per decode launch
           "prefix_kernel_ms": pfx_ms / max(1, n_dec) if n_pfx else None, "prefix_launches": n_pfx,
           "achieved_over": "lut_fast_kernel + its lut_prefix_kernel stages per launch" if n_pfx else kname,
           "algorithmic_bytes_per_launch": onchip_per_frame * per_launch,
           "lookups_per_frame": lookups,
           "algorithmic": f"{lookups} f/g table lookups per frame ({paths} path(s) x {info['lookups_per_path']}, the "
                          f"reference traversal of this code) x {ONCHIP_BYTES_PER_LOOKUP} B (SURVEY.md §8(d)) x "
                          f"{per_launch:.0f} frames per launch",
           # the lookups are ds_bpermute (a cross-lane crossbar read, ~40 % of ds_read_b32 when probed);
           # LDS-resident tables read with ds_read_b32/_b64 measured 5 % slower (profiles/r03k_ab_lds_tables.txt)
           "peak_probe": peaks, "frac_vs_probed_ds_bpermute": achieved / peaks["ds_bpermute_b32"],
           "peak_guide": {"ds_read_b32": GUIDE_LDS_B32_GBS, "ds_read_b64": GUIDE_LDS_B64_GBS},
           "lds_hit": kc.get("lds_hit"),
           "valu": valu_ceiling(kc),
           # traffic / lds_hit / valu / hbm.achieved_counters come from this committed PMC record
           # (profiles/counters.json, tools/counters.py), not from this run's counters
           "counters_record": {"file": "profiles/counters.json", "key": rec_id,
                               "sources": (rec or {}).get("sources")} if rec else None,
           "traffic_bytes_per_frame": (kc.get("traffic") / per_launch) if kc.get("traffic") else None,
           "traffic_note": "HBM-side bytes per launch of this kernel, 2 x FETCH_SIZE + WRITE_SIZE from separate "
                           "rocprofv3 --pmc passes (profiles/counters.json via tools/counters.py)",
           "hbm": {"achieved": hbm_bytes / (call_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": hbm_bytes / (call_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "call_ms": call_ms,
                   "pre_kernel_ms": pre_ms / max(1, n_pre), "algorithmic_bytes_per_call": hbm_bytes,
                   "traffic": (kc.get("traffic") or 0) + ((rec or {}).get("kernels", {}).get("root_pre_kernel", {})
                                                          .get("traffic") or 0) or None}}
    # the rocprof-measured HBM rate of the decode kernel: its PMC traffic per launch (counters.json)
    # over its launch duration timed here (HIP events)
    if kc.get("traffic"):
        kt_s = dec_ms / max(1, n_dec) * 1e-3
        out["hbm"]["achieved_counters"] = kc["traffic"] / kt_s / 1e9
        out["hbm"]["frac_counters"] = out["hbm"]["achieved_counters"] / HBM_PEAK_GBS
        out["hbm"]["counters_note"] = (f"{kname} HBM-side bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, rocprofv3 PMC "
                                       "passes) / its average launch duration from the HIP events")
    return out


def e2e_rate(args, ctx, wl):
    """Monte-Carlo rate of generate + decode + count over this rank's next
    frames (one step = args.frames new frames), all-reduced like run_rank."""
    import torch
    import torch.distributed as dist

    dec, src = wl.dec, wl.src
    prof = _has_prof(dec) and ctx._cuda
    state = {"f0": wl.frame0 + (1 << 40)}  # frames never decoded by the throughput loop
    acc = torch.zeros(2, dtype=torch.int64, device=ctx.device)

    fused = getattr(src, "decode_frames", None)  # qpd_mc_decode: generation feeds the decode kernel

    def step():
        if fused is not None:  # counters accumulated on the device by the same call
            fused(state["f0"], args.frames, counts=acc)
        else:  # a frame source without the fused call (the CPU tests' stand-in)
            msg, sym = src(state["f0"], args.frames)
            e = (dec.decode_batch(sym) != msg).sum(1)
            acc[0] += e.sum()
            acc[1] += (e > 0).sum()
        state["f0"] += args.frames

    if prof:
        dec.profile(True)
    _, wall = timed_steps(ctx, step, args.steps, 1)
    kt = dec.kernel_times() if prof else {}
    if prof:
        dec.profile(False)
    tmax = torch.tensor([wall], dtype=torch.float64, device=ctx.device)
    ctx.allreduce(tmax, dist.ReduceOp.MAX)
    frames = args.frames * args.steps * ctx.world
    r = {"value": frames / float(tmax.item()), "unit": "frames/s", "ms_per_step": float(tmax.item()) / args.steps * 1e3,
         "what": "per step: qpd_mc_decode (Philox msg, encode, BPSK+AWGN, channel quantizer writing the decoder's root "
                 "pre-pass rows, then the decode kernel) + error count"}
    if kt:
        mc_ms, n_mc = kt["mc"]
        r["mc_kernel_ms"] = mc_ms / max(1, n_mc)
        r["mc_kernel_bytes"] = args.frames * (args.N + 2 * dec.out_bits)  # pre-pass rows (N B) + msg (K B) + bits
        r["mc_kernel_gbs"] = r["mc_kernel_bytes"] / (r["mc_kernel_ms"] * 1e-3) / 1e9
    return r


def mc_rank(args, ctx, wl):
    """BASELINE config 5: one Monte-Carlo point of args.mc_frames frames sharded
    over the ranks (montecarlo.run_point; counters all-reduced over RCCL)."""
    import torch
    import torch.distributed as dist

    from quantized_decoder_polar_codes_amd import montecarlo as MC

    F = int(args.mc_frames)
    stop = args.mc_stop if args.mc_stop > 0 else None
    dec = wl.dec
    ctx.barrier()
    t0 = time.perf_counter()
    gloo = ctx.group is not None and dist.get_backend(ctx.group) == "gloo"
    r = MC.run_point(wl.src, dec.decode_batch, dec.K, args.ebn0, args.frames, F, stop, A=dec.out_bits,
                     gen_decode=getattr(wl.src, "decode_frames", None),
                     group=ctx.group, count_device="cpu" if gloo else ctx.device)
    ctx.barrier()
    tmax = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=ctx.device)
    ctx.allreduce(tmax, dist.ReduceOp.MAX)
    wall = float(tmax.item())
    if ctx.rank != 0:
        return None
    return {"metric": "Monte-Carlo frames/sec (generate + decode + count), N=1024 SCL-LUT L=8 Q=16; BER/BLER",
            "value": r.frames_decoded / wall, "unit": "frames/s", "n_gpus": ctx.world, "higher_is_better": True,
            "scaling": "strong", "wall_s": wall, "frames_decoded": r.frames_decoded, "blocks": r.blocks,
            "ber": r.ber, "bler": r.bler, "bit_errors": r.bit_errors, "block_errors": r.block_errors,
            "stopped_early": r.stopped_early, "dtype": "u8", "data": "synthetic (qpd_mc_frames, Philox keyed by "
            "global frame id: identical frames and counters at any rank count)",
            "config": {"workload": f"{args.kind} N={args.N} K={args.K}{(' L=' + str(args.L)) if 'SCL' in args.kind else ''} Q=16 Monte-Carlo point",
                       "ebn0_db": args.ebn0, "mc_frames": F, "stop_rule": f"Nblkerrs > {stop}" if stop else "none "
                       "(MaxBlock branch)", "batch_per_rank": args.frames, "luts": args.luts,
                       "parallelism": f"dp{ctx.world} (frames sharded by global frame id, RCCL counter all-reduce)"}}


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
    import shutil
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
    shutil.rmtree(tmp, ignore_errors=True)
    wall = max(walls)
    return {"value": total / wall, "unit": "frames/s", "cores": workers, "kind": kind,
            "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count(),
            "cores_note": f"{workers} worker processes = this GPU's CPU share (OMP_NUM_THREADS on the GPU box); "
                          f"the machine shows {os.cpu_count()} CPUs shared by its 8 GPUs",
            "build": ("reference decoder sources compiled by oracle/build_ref.sh: g++ -O3 -DNDEBUG, the reference's "
                      "Release flags without its -march=native (built in the container, run on this host)")
            if kind == "reference" else
            ("the oracle's C++ restatement of the reference (oracle/qpd_oracle.cpp, built by oracle/Makefile; "
             "oracle/_ref was not present on this host)"),
            "sample": f"{total} frames of the same workload (rank 0's first frames), {workers} worker processes x "
                      f"one decode() call per frame, {wall:.1f} s"}, outs


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or "unknown"


def rank_job(args, ctx, make_workload):
    """Everything one rank runs: its workload (global frames [r*F, (r+1)*F) of
    one Philox stream), then the throughput steps and the end-to-end rate, or
    the Monte-Carlo point.  Returns (rank 0's result dict or None, workload)."""
    wl = make_workload(ctx.rank * args.frames, 0 if args.mc_frames else args.frames)
    ctx.sync()
    if args.mc_frames:
        return mc_rank(args, ctx, wl), wl
    res = run_rank(args, ctx, wl)
    if not args.no_e2e:
        e2e = e2e_rate(args, ctx, wl)
        if res is not None:
            res["monte_carlo_e2e"] = e2e
    return res, wl


def parity_and_baseline(args, wl, res):
    """Rank 0: the reference CPU decoder on a bounded sample of this rank's
    resident frames (cpu_baseline) and the GPU bits of the same frames against
    it (parity_sample).  Runs after the timed steps at any world size, so every
    line of a 1..8-GPU scaling run carries its bit-exactness check."""
    workers = args.cpu_workers or min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)))
    sample = wl.sym[: 1 << 15].cpu().numpy()
    cb, parts = cpu_baseline(args, wl.packed, wl.fm, wl.nt, sample, args.cpu_baseline_seconds, max(1, workers),
                             wl.dec.out_bits)
    res["cpu_baseline"] = cb
    gpu_out = wl.dec.decode_batch(wl.sym[: 1 << 15]).cpu().numpy()
    ok = all(np.array_equal(gpu_out[o:o + len(r)], r) for o, r in parts)
    res["parity_sample"] = {"frames": int(sum(len(r) for _, r in parts)), "bit_exact_vs_" + cb["kind"]: bool(ok),
                            "rank": 0, "frames_from": "rank 0's first resident frames (global ids 0..)"}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args, argv))
    import torch
    import torch.distributed as dist

    launched = "WORLD_SIZE" in os.environ  # under torch.distributed.run (the driver's N-GPU launches)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal of the N-rank path on fewer GPUs (tests of the launch and
    # sharding on a one-GPU box): QPD_BENCH_DEVICES maps local ranks onto the
    # listed devices, QPD_BENCH_BACKEND=gloo replaces RCCL (which refuses two
    # ranks on one device).  Defaults: rank i on GPU i, RCCL.
    devs = [int(x) for x in os.environ.get("QPD_BENCH_DEVICES", "").split(",") if x.strip()]
    torch.cuda.set_device(devs[local % len(devs)] if devs else (local if world > 1 else 0))
    group = None
    if launched:  # every torchrun launch, world size 1 included, reduces over a process group
        dist.init_process_group(os.environ.get("QPD_BENCH_BACKEND", "nccl"))  # "nccl" = RCCL over xGMI
        group = dist.group.WORLD
    dev = torch.device("cuda", torch.cuda.current_device())
    ctx = Ctx(rank, world, dev, group)

    def make(frame0, frames):
        return workload(args.N, args.K, args.L, args.kind, frames, args.ebn0, args.luts, args.design_snr,
                        frame0=frame0, device=dev.index, max_waves=args.max_waves, engine=args.engine)

    res, wl = rank_job(args, ctx, make)
    if not args.mc_frames and not args.no_cpu_baseline:
        if res is not None:
            parity_and_baseline(args, wl, res)
            res["config"]["process_group"] = dist.get_backend(group) if group is not None else None
        if group is not None:
            dist.barrier(group=group)  # the other ranks wait for rank 0's CPU leg
    if res is not None:
        print(json.dumps(res), flush=True)
    if group is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
