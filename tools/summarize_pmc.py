"""Summarize SQ counter passes for the decode kernel: totals and per-frame."""
import collections
import csv
import sys

frames = float(sys.argv[1])
for path in sys.argv[2:]:
    agg = collections.defaultdict(float)
    nd = set()
    for r in csv.DictReader(open(path)):
        kn = r["Kernel_Name"]
        if ("lut_fast_kernel" in kn and "true>(" not in kn.replace(" ", "")) or "lut_decode_kernel" in kn:  # not the prefix
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            nd.add(r["Dispatch_Id"])
    print(f"# {path} ({len(nd)} dispatch(es))")
    for k in sorted(agg):
        v = agg[k] / max(1, len(nd))
        print(f"{k:24s} {v:18.0f}   per frame {v / frames:12.1f}")
