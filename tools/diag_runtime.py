"""Diagnostic: which HIP runtime does libqpd.so bind to, and can it decode?
usage: python tools/diag_runtime.py [torch_first|lib_first]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
mode = sys.argv[1] if len(sys.argv) > 1 else "torch_first"
if mode == "torch_first":
    import torch

    print("torch.cuda.is_available", torch.cuda.is_available(), flush=True)
L = ctypes.CDLL(os.path.join(ROOT, "quantized_decoder_polar_codes_amd", "libqpd.so"))
maps = open("/proc/self/maps").read()
print(sorted(set(l.split()[-1] for l in maps.splitlines() if "amdhip" in l or "hsa-runtime" in l)), flush=True)
import quantized_decoder_polar_codes_amd as Q  # noqa: E402
from quantized_decoder_polar_codes_amd import codes as C, lut as LU  # noqa: E402

N, K = 16, 8
_, mb, fm, mm = C.construct_pw(N, K)
d = Q.from_packed("SC-LUT", LU.minsum_uniform_luts(N), K, fm, device=0)
print(d.info(), flush=True)
sym = np.random.default_rng(0).integers(0, 16, size=(4, N), dtype=np.int32)
print(d.decode_batch(sym), flush=True)
print("OK", mode)
