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
        args = kn.split("lut_fast_kernel<", 1)[1].split(">", 1)[0].replace(" ", "").split(",") if "lut_fast_kernel<" in kn else []
        if (args and not (len(args) >= 5 and args[4] == "true")) or "lut_decode_kernel" in kn:  # not the prefix (PFX)
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            nd.add(r["Dispatch_Id"])
    print(f"# {path} ({len(nd)} dispatch(es))")
    for k in sorted(agg):
        v = agg[k] / max(1, len(nd))
        print(f"{k:24s} {v:18.0f}   per frame {v / frames:12.1f}")
