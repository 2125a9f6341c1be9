"""Diagnostic: how many of the list paths' f / g rows an op could share (the
"shared-lineage row written once per owning path" slab design).
The host engine computes a path's S[d+1] only when no earlier path has the same
inputs (the same S[d] source and, for g, the same U[d+1] source); counted here per
depth on the bench workload (MinDistortion tables, 2 dB).  CPU only.
usage: python tools/row_sharing.py [frames] [L]"""
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

SRC = r'''
#include <cstdio>
#include <cstdint>
static long g_rows[2][2][20];  // [shared][isg][depth]
#define QPD_HOST_FG_HOOK(d, isg, shared) (++g_rows[(shared) ? 1 : 0][(isg) ? 1 : 0][d])
#include "qpd_host.hpp"
extern "C" void rs_run(const qpd_config *c, const int32_t *in, int64_t B, long *out) {
    std::unique_ptr<qpd_host::Plan> p = qpd_host::make_plan(c);
    qpd_host::Engine<uint8_t> e(*p);
    std::vector<uint8_t> o(p->out_k);
    for (int64_t b = 0; b < B; ++b) e.decode(in + b * p->N, o.data());
    for (int i = 0; i < 80; ++i) out[i] = (&g_rows[0][0][0])[i];
}
'''
so, cpp = "/tmp/row_sharing.so", "/tmp/row_sharing.cpp"
open(cpp, "w").write(SRC)
subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-I", f"{ROOT}/include", "-I",
                f"{ROOT}/quantized_decoder_polar_codes_amd/csrc", cpp, "-o", so], check=True)
lib = ctypes.CDLL(so)
N, K = 1024, 512
F = int(sys.argv[1]) if len(sys.argv) > 1 else 16
L = int(sys.argv[2]) if len(sys.argv) > 2 else 8
_, mb, fm, mm = C.construct_pw(N, K)
d = LG.design(N, 16, 3.0)
sigma = MC.sigma_for(2.0, K / N)
_, _, edges, clut = LG.channel_quantizer(sigma, 128, 16)
_, sym, _ = ref_frames(N, K, mb, 1234, 0, F, sigma, edges, clut, 16)
dec = D.from_packed("SCL-LUT", d.packed(), K, fm, L=L, create=False)
sym = np.ascontiguousarray(sym, dtype=np.int32)
out = np.zeros(80, np.int64)
lib.rs_run(ctypes.byref(dec._cfg), sym.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(F),
           out.ctypes.data_as(ctypes.c_void_p))
g = out.reshape(2, 2, 20)
print(f"SCL-LUT N={N} K={K} L={L}, {F} frames: path rows of f / g ops (computed + shared) per depth d -> d+1")
for dd in range(0, 10):
    for isg, nm in ((0, "f"), (1, "g")):
        comp, sh = g[0, isg, dd], g[1, isg, dd]
        if comp + sh:
            print(f"  d={dd} {nm}: rows {comp + sh:8d}  shared {sh / (comp + sh):6.3f}")
tot = g[:, :, 0:4].sum()
print(f"  depths 0-3 (the slab's S[1..4] rows): shared {g[1, :, 0:4].sum() / max(1, tot):.3f} of {tot}")
