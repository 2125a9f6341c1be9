"""Tuning sweep (one process): frames/s of the decode kernel across LDS budgets,
batch sizes and grid caps.  usage: python tools/sweep.py [kind] [N K L]"""
import itertools
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import quantized_decoder_polar_codes_amd as Q  # noqa: E402
from quantized_decoder_polar_codes_amd import codes as C, lut as LU  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "SCL-LUT"
N, K, L = (int(x) for x in sys.argv[2:5]) if len(sys.argv) > 4 else (1024, 512, 8)
budgets = [int(x) for x in os.environ.get("SWEEP_BUDGETS", "8192,12288,16384,24576,32768").split(",")]
frames_list = [int(x) for x in os.environ.get("SWEEP_FRAMES", "65536,262144").split(",")]
waves_list = [int(x) for x in os.environ.get("SWEEP_WAVES", "0").split(",")]
import bench  # noqa: E402

# the bench's workload (MinDistortion tables and channel quantizer, GPU frames at Eb/N0 2 dB)
maxF = max(frames_list)
_wl = bench.workload(N, K, L, kind, maxF, float(os.environ.get("SWEEP_EBN0", "2.0")),
                     os.environ.get("SWEEP_LUTS", "mindistortion"))
packed, fm, nt, sym = _wl.packed, _wl.fm, _wl.nt, _wl.sym
p = packed
ref = None
for budget, F, mw in itertools.product(budgets, frames_list, waves_list):
    os.environ["QPD_LDS_BUDGET"] = str(budget)
    d = Q.from_packed(kind, p, K, fm, L=L, node_type=nt, max_waves=mw)
    info = d.info()
    x = sym[:F]
    out = d.decode_batch(x)
    torch.cuda.synchronize()
    if ref is None or ref.shape[0] < F:
        ref = out.clone()
    assert torch.equal(out[: min(F, ref.shape[0])], ref[: min(F, ref.shape[0])])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 3
    e0.record()
    for _ in range(reps):
        d.decode_batch(x)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"{kind} N={N} L={L} budget={budget:6d} lds_from={info['lds_from_depth']} lds={info['lds_bytes_per_wave']:6d} "
          f"frames={F:7d} max_waves={info['max_waves']:5d}  {ms:8.3f} ms  {F / ms * 1e3 / 1e6:8.3f} Mframes/s", flush=True)
    del d
