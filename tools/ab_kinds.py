"""A/B timing of one libqpd build (QPD_LIB=...) on the bench workload of several decoders.
Prints Mframes/s and a digest of the decoded bits (equal digests across builds = same output).
usage: QPD_LIB=build_variants/libqpd_X.so python tools/ab_kinds.py [kind[:L] ...]"""
import hashlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

kinds = sys.argv[1:] or ["SCL-LUT", "FastSCL-LUT"]
F = int(os.environ.get("AB_FRAMES", "1048576"))
for spec in kinds:
    kind, L = (spec.split(":") + ["8"])[:2]
    wl = bench.workload(1024, 512, int(L), kind, F, 2.0, max_waves=int(os.environ.get("QPD_MAX_WAVES", "0")))
    d, sym = wl.dec, wl.sym
    out = d.decode_batch(sym)
    torch.cuda.synchronize()
    dig = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:12]
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        d.decode_batch(sym)
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    tag = os.environ.get("AB_TAG") or os.path.basename(os.environ.get("QPD_LIB", "libqpd.so"))
    print(f"{tag:30s} {spec:12s} {best:8.3f} ms "
          f"{F / best / 1e3:8.3f} Mframes/s digest {dig}", flush=True)
