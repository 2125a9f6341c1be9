"""Repeat one GPU-vs-oracle parity case many times and report which frames differ per run
(diagnosis of run-to-run differences; QPD_LIB=... selects the build).
usage: python tools/diag_repro.py KIND N K L TABLES [reps]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402  (the checker)

import quantized_decoder_polar_codes_amd as Q  # noqa: E402
from quantized_decoder_polar_codes_amd import codes as C  # noqa: E402
from quantized_decoder_polar_codes_amd import lut as LU  # noqa: E402

KINDS = ["SC-LUT", "SCL-LUT", "FastSC-LUT", "FastSCL-LUT"]
kind, N, K, L, tables = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 20
seed = 1000 + N + 7 * L + KINDS.index(kind)
if tables == "minsum":
    p = LU.minsum_uniform_luts(N)
elif tables == "continuous":
    p = LU.random_luts(N, 16, seed=seed, distinct_mags=None)
else:
    p = LU.random_luts(N, 16, seed=seed, distinct_mags=3, per_element=(tables == "perelem"))
_, mb, fm, mm = C.construct_pw(N, K)
nt = C.identify_nodes(N, mb).astype(np.int32)
B = 24 if N >= 1024 and kind in ("SCL-LUT", "FastSCL-LUT") else 200
sym = np.random.default_rng(seed).integers(0, 16, size=(B, N), dtype=np.int32)
want = oracle.decode_lut(kind, p, K, L, fm, sym, node_type=nt)
tag = os.environ.get("QPD_LIB", "libqpd.so")
dec = Q.from_packed(kind, p, K, fm, L=L, node_type=nt)
print(tag, kind, N, K, L, tables, "engine", dec.info()["engine"], flush=True)
for r in range(reps):
    if r % 2:
        dec = Q.from_packed(kind, p, K, fm, L=L, node_type=nt)
    got = dec.decode_batch(sym)
    bad = np.flatnonzero((got != want).any(1))
    one = [int(np.flatnonzero((dec.decode_batch(sym[i:i + 1])[0] != want[i]).astype(np.int8)).size) for i in bad[:3]]
    print(f"rep {r}: {bad.size} frames differ {bad[:8].tolist()} (alone: bits differing {one})", flush=True)
