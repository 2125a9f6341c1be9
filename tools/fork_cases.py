"""Diagnostic: survivor-selection cases of the SCL-LUT info-leaf forks on the
bench workload (MinDistortion tables at 3 dB, the driver's channel at 2 dB),
per frame and per wave of 8 frames (the GPU kernel's identity fast path needs
all 8 frames of a wave to qualify).  CPU only (host engine + numpy frames)."""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from mc_ref import frames as ref_frames  # noqa: E402
from quantized_decoder_polar_codes_amd import codes as C, decoders as D, lutgen as LG, montecarlo as MC  # noqa: E402

so = "/tmp/fork_cases.so"
subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-I", f"{ROOT}/include", "-I",
                f"{ROOT}/quantized_decoder_polar_codes_amd/csrc", f"{ROOT}/tools/fork_cases.cpp", "-o", so], check=True)
lib = ctypes.CDLL(so)
N, K = 1024, 512
L = int(sys.argv[3]) if len(sys.argv) > 3 else 8
F = int(sys.argv[1]) if len(sys.argv) > 1 else 64
ebn0 = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
_, mb, fm, mm = C.construct_pw(N, K)
d = LG.design(N, 16, 3.0)
sigma = MC.sigma_for(ebn0, K / N)
_, _, edges, clut = LG.channel_quantizer(sigma, 128, 16)
_, sym, _ = ref_frames(N, K, mb, 1234, 0, F, sigma, edges, clut, 16)
dec = D.from_packed("SCL-LUT", d.packed(), K, fm, L=L, create=False)
sym = np.ascontiguousarray(sym, dtype=np.int32)
cases = np.zeros(F * K, np.int32)
per = np.zeros(F, np.int64)
n = lib.fc_run(ctypes.byref(dec._cfg), sym.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(F),
               cases.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(len(cases)), per.ctypes.data_as(ctypes.c_void_p))
raw = cases[:n].reshape(F, -1)  # every frame forks at the same info leaves
strict = (raw // 1000) % 2 == 1
tie = raw >= 2000
c = raw % 10
below = (raw // 10) % 10
unsorted = (raw // 100) % 10 == 1
print(f"  L={L}: strict identity {strict.mean():.3f}, tie among the first L ranks {tie.mean():.3f}")
print("  flips below the largest keep (per fork):", {int(b): round(float(np.mean(below == b)), 3) for b in range(10)})
print("  keeps not in stable order:", round(float(unsorted.mean()), 3))
print(f"frames {F}, info-leaf forks per frame {c.shape[1]}")
for k, name in enumerate(("identity", "one swap", "other")):
    print(f"  per frame: {name:9s} {np.mean(c == k):.3f}")
w = c[: (F // 8) * 8].reshape(-1, 8, c.shape[1])
ident = (w == 0).all(1).mean()
ident_or_swap = (w <= 1).all(1).mean()
print(f"  per wave of 8 frames: identity {ident:.3f}, identity-or-one-swap {ident_or_swap:.3f}, "
      f"full selection {1 - ident_or_swap:.3f} (now {1 - ident:.3f})")
