#!/usr/bin/env python3
"""Throughput of the float64-LLR decoders on one MI355X,
beside the reference decoder on the host (oracle/_ref, one decode() per frame).

A step = one qpd_decode_f64 launch over F frames of AWGN LLRs already resident
in HBM (generated on the host with numpy, copied before timing: the reference
drivers' channel, mainFPDecoder.py / mainQuantizedDecoder_ContinuousDomain.py).
Prints one JSON line per decoder kind.  Not the headline bench (bench.py is);
this is the measurement leg of row F4.

  python tools/bench_float.py --kinds SCL,FastSCL --N 1024 --K 512 --L 8
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kinds", default="SC,SCL,CA-SCL,FastSC,FastSCL,SC-Uniform,SCL-Uniform,SC-Lloyd,SCL-Lloyd")
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--K", type=int, default=512)
    ap.add_argument("--L", type=int, default=8)
    ap.add_argument("--frames", type=int, default=1 << 15)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--ebn0", type=float, default=2.0)
    ap.add_argument("--cpu-seconds", type=float, default=3.0)
    args = ap.parse_args()

    import torch

    import oracle
    from quantized_decoder_polar_codes_amd import codes as C
    from quantized_decoder_polar_codes_amd import montecarlo as MC
    from quantized_decoder_polar_codes_amd.decoders import from_quant
    from test_float_oracle import CRC24, quant_for, ref_decoder

    torch.cuda.set_device(0)
    N, K, L = args.N, args.K, args.L
    _, mb, fm, mm = C.construct_pw(N, K)
    nt = C.identify_nodes(N, mb).astype(np.int32)
    sigma = MC.sigma_for(args.ebn0, K / N)
    rng = np.random.default_rng(77)
    msg = rng.integers(0, 2, size=(args.frames, K), dtype=np.uint8)
    x = C.polar_encode(msg, mb, N)
    llr = 2 * ((1.0 - 2.0 * x) + sigma * rng.standard_normal((args.frames, N))) / sigma ** 2
    d_llr = torch.from_numpy(llr).cuda()
    d_msg = torch.from_numpy(msg).cuda()
    R = oracle.reference_module()
    for kind in args.kinds.split(","):
        q = quant_for(kind, N, sigma=sigma)
        kw = dict(A=K - 24, crc_n=24, crc_loc=CRC24) if kind == "CA-SCL" else {}
        lst = kind in ("SCL", "CA-SCL", "FastSCL", "SCL-Uniform", "SCL-Lloyd")
        dec = from_quant(kind, N, K, fm, L=L, node_type=nt, quant=q, **kw)
        out = dec.decode_batch(d_llr)
        torch.cuda.synchronize()
        stream = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(args.steps):
            out = dec.decode_batch(d_llr)
        e1.record(stream)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        kern_ms = e0.elapsed_time(e1) / args.steps
        ob = dec.out_bits
        err = (out != d_msg[:, :ob])
        res = {"kind": kind, "N": N, "K": K, "L": L if lst else 1, "frames_per_step": args.frames,
               "frames_per_s": args.frames * args.steps / wall, "kernel_ms": kern_ms, "ebn0_db": args.ebn0,
               "ber": float(err.float().mean().item()), "bler": float(err.any(1).float().mean().item()),
               "engine": "generic", "info": {k: v for k, v in dec.info().items() if k in ("max_waves",
                                                                                        "scratch_bytes_per_wave")}}
        if R is not None and hasattr(R, "SCLDecoder"):
            A, crc = (K - 24, (24, CRC24)) if kind == "CA-SCL" else (None, None)
            rd = ref_decoder(R, kind, N, K, L if lst else 1, fm.tolist(), mm.tolist(), nt.tolist(), q, A, crc)
            got, t0 = [], time.perf_counter()
            while time.perf_counter() - t0 < args.cpu_seconds and len(got) < args.frames:
                got.append(rd.decode(llr[len(got)][None]))
            dt = time.perf_counter() - t0
            g = out[: len(got)].cpu().numpy()
            res["cpu_baseline"] = {"frames_per_s": len(got) / dt, "cores": 1, "kind": "reference",
                                   "sample": f"{len(got)} frames, one decode() per frame"}
            res["parity_sample"] = {"frames": len(got), "bit_exact_vs_reference": bool(np.array_equal(np.stack(got), g))}
        print(json.dumps(res), flush=True)
        del dec


if __name__ == "__main__":
    main()
