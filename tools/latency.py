"""Per-frame latency of the drop-in decode() path, called the way the
reference drivers call it: one frame per call from a Python loop
(mainQuantizedDecoder_LLRDomain.py:178).  Each call copies the frame to the
device, runs the decode kernel(s) on one frame and copies K bytes back
(qpd_decode_host; synchronous).  Prints one JSON line per configuration.

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
    for kind, N, K, L in (("SCL-LUT", 1024, 512, 8), ("FastSCL-LUT", 1024, 512, 8), ("SC-LUT", 128, 32, 1),
                          ("SC-LUT", 1024, 512, 1)):
        wl = bench.workload(N, K, L, kind, frames, 2.0)
        sym = wl.sym.cpu().numpy()
        dec = wl.dec
        for i in range(5):  # warm-up (first call builds the staging buffers)
            dec.decode(sym[i])
        t = []
        for i in range(frames):
            t0 = time.perf_counter()
            out = dec.decode(sym[i])
            t.append(time.perf_counter() - t0)
        ref = dec.decode_batch(sym)
        assert np.array_equal(out, ref[frames - 1]), "single-frame decode differs from the batched one"
        t = np.array(t) * 1e3
        print(json.dumps({"kind": kind, "N": N, "K": K, "L": L, "calls": frames, "ms_p50": float(np.median(t)),
                          "ms_p90": float(np.percentile(t, 90)), "ms_min": float(t.min()),
                          "frames_per_s_one_call_per_frame": float(1e3 / np.median(t))}), flush=True)


if __name__ == "__main__":
    main()
