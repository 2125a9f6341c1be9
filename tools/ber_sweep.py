"""BER / BLER curve of the bench decoder on the GPU, the way the reference's
driver produces it (mainQuantizedDecoder_LLRDomain.py:130-203): per Eb/N0 the
driver's MinDistortion channel quantizer (lutgen.channel_quantizer), decoder
tables designed once at 3 dB, and the driver's stop rule (Nblkerrs > 1000, else
MaxBlock).  Frames, decode and counters run on the GPU (montecarlo.run_point
with the fused qpd_mc_decode path).

At every point a sample of the same frames is also decoded by the reference
decoder itself (oracle/_ref, compiled from its sources; test infrastructure,
run beside the product here): the bits must be equal, so the point's BER/BLER
are the reference's on those frames ("BER match", BASELINE.json metric).

usage (GPU box): python tools/ber_sweep.py [--kind SCL-LUT] [--ebn0 0,1,2,3,4,5]
One JSON line per point.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="SCL-LUT", choices=bench.KINDS)
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--K", type=int, default=512)
    ap.add_argument("--L", type=int, default=8)
    ap.add_argument("--ebn0", default="0,1,2,3,4,5")
    ap.add_argument("--max-blocks", type=float, default=1e8)
    ap.add_argument("--stop", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--check", type=int, default=400, help="frames per point decoded by the reference too")
    args = ap.parse_args()

    import torch

    from latency import reference_decoder
    from quantized_decoder_polar_codes_amd import lutgen as LG
    from quantized_decoder_polar_codes_amd import montecarlo as MC

    wl = bench.workload(args.N, args.K, args.L, args.kind, 0, 2.0)
    dec = wl.dec
    ref = reference_decoder(args.kind, wl)
    rate = (dec.out_bits if args.kind.startswith("CA-") else dec.K) / dec.N
    for eb in (float(x) for x in args.ebn0.split(",")):
        sigma = MC.sigma_for(eb, rate)
        _, _, edges, clut = LG.channel_quantizer(sigma, 128, 16)
        src = MC.GpuFrames(dec, edges, clut, 16, sigma, seed=MC.point_seed(2024, eb))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = MC.run_point(src, dec.decode_batch, dec.K, eb, args.batch, int(args.max_blocks), args.stop,
                           A=dec.out_bits, count_device=src.device, gen_decode=src.decode_frames)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        rec = {"kind": args.kind, "N": dec.N, "K": dec.K, "L": args.L, "ebn0_db": eb, "ber": res.ber, "bler": res.bler,
               "blocks": res.blocks, "bit_errors": res.bit_errors, "block_errors": res.block_errors,
               "frames_decoded": res.frames_decoded, "stopped_early": res.stopped_early, "seconds": dt,
               "frames_per_s": res.frames_decoded / dt}
        if ref is not None and args.check > 0:
            msg, sym = src(0, args.check)  # the point's first frames
            bits = dec.decode_batch(sym).cpu().numpy()
            s = sym.cpu().numpy()
            rbits = np.stack([np.asarray(ref.decode(s[i][None])).reshape(-1) for i in range(args.check)])
            m = msg.cpu().numpy()
            rec["reference_check"] = {"frames": args.check, "bits_equal": bool(np.array_equal(bits, rbits)),
                                      "block_errors_gpu": int((bits != m).any(1).sum()),
                                      "block_errors_reference": int((rbits != m).any(1).sum())}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
