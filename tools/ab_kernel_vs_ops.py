"""Diagnosis: the FastSCL-LUT kernel on the SCL-LUT op mix.  FastSCL-LUT with no
special nodes (node_type all -1) decodes like SCL-LUT, with the same op list
but compiled into the FastSCL-LUT instantiation; compared with SCL-LUT on the
SCL-LUT instantiation without the frozen-prefix stages (QPD_NO_PFX=1), the
difference is the kernel's code, not the schedule.  Prints Mframes/s."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import quantized_decoder_polar_codes_amd as Q  # noqa: E402

F = int(os.environ.get("AB_FRAMES", "1048576"))
wl = bench.workload(1024, 512, 8, "SCL-LUT", F, 2.0)


def rate(d):
    out = d.decode_batch(wl.sym)
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        d.decode_batch(wl.sym)
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return F / best / 1e3, out


os.environ["QPD_NO_PFX"] = "1"
r1, o1 = rate(Q.from_packed("SCL-LUT", wl.packed, 512, wl.fm, L=8))
nt = -np.ones(2 * 1024 - 1, dtype=np.int32)
r2, o2 = rate(Q.from_packed("FastSCL-LUT", wl.packed, 512, wl.fm, L=8, node_type=nt))
del os.environ["QPD_NO_PFX"]
r3, _ = rate(Q.from_packed("FastSCL-LUT", wl.packed, 512, wl.fm, L=8, node_type=wl.nt))
print(f"SCL-LUT kernel, SCL ops (no prefix)        {r1:8.3f} Mframes/s")
print(f"FastSCL-LUT kernel, SCL ops (no specials)  {r2:8.3f} Mframes/s")
print(f"FastSCL-LUT kernel, FastSCL ops            {r3:8.3f} Mframes/s")
