"""Diagnostic: how many survivor-selection layers the FastSCL-LUT rate-1 (R1)
nodes run before their selection becomes the identity, per frame and per wave
of 8 frames (the kernel stops a wave's R1 node at the first layer where all
its frames' selections are the identity), on the bench workload.  CPU only
(host engine + numpy frames)."""
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

so = "/tmp/r1_layers.so"
subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-I", f"{ROOT}/include", "-I",
                f"{ROOT}/quantized_decoder_polar_codes_amd/csrc", f"{ROOT}/tools/r1_layers.cpp", "-o", so], check=True)
lib = ctypes.CDLL(so)
N, K, L = 1024, 512, 8
F = int(sys.argv[1]) if len(sys.argv) > 1 else 64
ebn0 = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
_, mb, fm, mm = C.construct_pw(N, K)
nt = C.identify_nodes(N, mb).astype(np.int32)
d = LG.design(N, 16, 3.0)
sigma = MC.sigma_for(ebn0, K / N)
_, _, edges, clut = LG.channel_quantizer(sigma, 128, 16)
_, sym, _ = ref_frames(N, K, mb, 1234, 0, F, sigma, edges, clut, 16)
dec = D.from_packed("FastSCL-LUT", d.packed(), K, fm, L=L, node_type=nt, create=False)
sym = np.ascontiguousarray(sym, dtype=np.int32)
rec = np.zeros(F * 64, np.int32)
n = lib.r1_run(ctypes.byref(dec._cfg), sym.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(F),
               rec.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(len(rec)))
r = rec[:n].reshape(F, -1)  # every frame has the same R1 nodes
temp, first = r // 100, r % 100
m = np.minimum(L - 1, temp)
print(f"frames {F}, R1 nodes per frame {r.shape[1]}, sizes {sorted(set(temp[0].tolist()))}")
print("  per frame: layers run (first identity layer, m if none):",
      {int(k): round(float(np.mean(first == k)), 3) for k in range(8)})
print("  per frame: mean layers run / m:", round(float(first.sum() / m.sum()), 3))
w = first[: (F // 8) * 8].reshape(-1, 8, r.shape[1]).max(1)  # a wave runs until all 8 frames are done
mw = m[: (F // 8) * 8].reshape(-1, 8, r.shape[1])[:, 0]
print("  per wave of 8 frames: layers run", {int(k): round(float(np.mean(w == k)), 3) for k in range(8)},
      "mean layers / m", round(float(w.sum() / mw.sum()), 3))
