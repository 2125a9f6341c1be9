"""Per-frame latency of the drop-in decode() path, called the way the
reference drivers call it: one frame per call from a Python loop
(mainQuantizedDecoder_LLRDomain.py:178), beside the reference decoder itself
(oracle/_ref, the same frames, one pybind11 decode() per frame, this host).
Two engines behind qpd_decode_host: the host engine (the default for a
per-frame call, csrc/qpd_host.hpp) and a one-frame GPU call (copy in, decode
kernel(s), copy out; set_host_engine("gpu")).  One JSON line per configuration.

usage (GPU box): python tools/latency.py [frames]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    for kind, N, K, L in (("SC-LUT", 128, 32, 1), ("SC-LUT", 1024, 512, 1), ("FastSC-LUT", 1024, 512, 1),
                          ("SCL-LUT", 1024, 512, 8), ("FastSCL-LUT", 1024, 512, 8)):
        wl = bench.workload(N, K, L, kind, frames, 2.0)
        sym = wl.sym.cpu().numpy()
        dec = wl.dec
        batch = dec.decode_batch(sym)
        rec = {"kind": kind, "N": N, "K": K, "L": L, "calls": frames,
               "host_max_frames_auto": int(dec.info()["host_max_frames"])}
        for mode in ("auto", "gpu"):
            dec.set_host_engine(mode)
            for i in range(5):  # warm-up (first call builds the staging buffers)
                dec.decode(sym[i])
            t, outs = [], []
            for i in range(frames):
                t0 = time.perf_counter()
                outs.append(dec.decode(sym[i]))
                t.append(time.perf_counter() - t0)
            assert np.array_equal(np.stack(outs), batch), f"{mode}: per-frame decode differs from the batched one"
            t = np.array(t) * 1e3
            rec[mode] = {"ms_p50": float(np.median(t)), "ms_p90": float(np.percentile(t, 90)), "ms_min": float(t.min())}
        dec.set_host_engine("auto")
        ref = reference_decoder(kind, wl)
        if ref is not None:
            n_ref = min(frames, 60 if L > 1 else frames)
            for i in range(3):
                ref.decode(sym[i][None])
            t, outs = [], []
            for i in range(n_ref):
                t0 = time.perf_counter()
                outs.append(ref.decode(sym[i][None]))
                t.append(time.perf_counter() - t0)
            t = np.array(t) * 1e3
            rec["reference"] = {"ms_p50": float(np.median(t)), "ms_min": float(t.min()), "calls": n_ref,
                                "bits_equal": bool(np.array_equal(np.stack(outs), batch[:n_ref]))}
        print(json.dumps(rec), flush=True)


def reference_decoder(kind, wl):
    """The reference's own class (oracle/_ref, compiled from its sources; test
    infrastructure, timed beside the product here), or None if not built."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    R = oracle.reference_module()
    if R is None:
        return None
    from quantized_decoder_polar_codes_amd import lut as LU

    fs, gs, vcl = LU.unpack_to_reference(wl.packed)
    N, K, L = wl.dec.N, wl.dec.K, wl.dec.L
    fz, mm = wl.fm.astype(int).tolist(), (1 - wl.fm).astype(int).tolist()
    return {"SC-LUT": lambda: R.SCLUTDecoder(N, K, fz, mm, fs, gs, vcl),
            "SCL-LUT": lambda: R.SCLLUTDecoder(N, K, L, fz, mm, fs, gs, vcl),
            "FastSC-LUT": lambda: R.FastSCLUTDecoder(N, K, fz, mm, wl.nt.tolist(), fs, gs, vcl),
            "FastSCL-LUT": lambda: R.FastSCLLUTDecoder(N, K, L, fz, mm, wl.nt.tolist(), fs, gs, vcl)}[kind]()


if __name__ == "__main__":
    main()
