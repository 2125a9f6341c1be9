"""Per-op-class wave cycles of the fast kernel (diagnostic build with -DQPD_STAMPS).
usage: QPD_LIB=build_variants/libqpd_stamps.so python tools/stamps.py [kind N K L frames]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import quantized_decoder_polar_codes_amd as Q  # noqa: E402
from quantized_decoder_polar_codes_amd import _lib, codes as C, lut as LU  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "SCL-LUT"
N, K, L, F = (int(x) for x in sys.argv[2:6]) if len(sys.argv) > 5 else (1024, 512, 8, 262144)
names = ["F", "G", "LEAF_L", "LEAF_R", "COMB", "R0", "R1", "REP", "SPC", "BOT3", "IMPORT", "EXPORT"]
import bench  # noqa: E402

_wl = bench.workload(N, K, L, kind, F, 2.0)  # the bench workload (MinDistortion, 2 dB)
d, fm, nt, sym = _wl.dec, _wl.fm, _wl.nt, _wl.sym
lib = _lib.load()
buf = (ctypes.c_ulonglong * 64)()
d.decode_batch(sym)
torch.cuda.synchronize()
lib.qpd_debug_stamps(buf)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
d.decode_batch(sym)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1)
lib.qpd_debug_stamps(buf)
acc = np.array(buf[:32], dtype=np.float64)
cnt = np.array(buf[32:], dtype=np.float64)
info = d.info()
tasks = (F + info["frames_per_wave"] - 1) // info["frames_per_wave"]
tot = acc.sum()
print(f"{kind} N={N} L={L} frames={F} waves={info['max_waves']} wall {ms:.3f} ms ({F / ms / 1e3:.3f} Mframes/s)")
print(f"total stamped wave-cycles per task {tot / tasks:,.0f}")
for c in range(32):
    if cnt[c] == 0:
        continue
    if os.environ.get("STAMPS_DEPTH"):
        nm = "TAIL" if c == 31 else (["F", "G", "COMB"][c // 8] + f" d{c % 8}" if c < 24 else
                                     {24: "BOT3", 25: "LEAF", 26: "R0", 27: "R1", 28: "REP", 29: "SPC", 30: "BOTX"}[c])
    else:
        nm = "TAIL" if c == 31 else ({24: "R1<=8", 25: "R1 9-16", 26: "R1>16"}[c] if 24 <= c <= 26 else
                                  names[c // 2] + ("/sync" if c % 2 else ""))
    print(f"  {nm:12s} ops/task {cnt[c] / tasks:8.1f}  cyc/op {acc[c] / cnt[c]:9.0f}  cyc/task {acc[c] / tasks:11,.0f}  "
          f"{100 * acc[c] / tot:5.1f}%")
