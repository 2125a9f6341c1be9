"""Fold rocprofv3 FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_traffic.json
(HBM-side bytes per launch of the decode kernel), keyed like bench.py's lookup.

usage: python tools/pmc_traffic.py KEY FETCH_CSV WRITE_CSV [KERNEL_SUBSTR]
FETCH_SIZE/WRITE_SIZE are in KiB per dispatch (memory-side L2 requests; the
Infinity Cache is counted, not excluded -- MI355X_MICROARCH.md §HBM).  Our
reads are not 16-B/lane streaming loads, so the x2 FETCH correction for that
pattern does not apply; the value is reported raw and marked uncalibrated."""
import csv
import json
import os
import sys

key, fcsv, wcsv = sys.argv[1:4]
sub = sys.argv[4] if len(sys.argv) > 4 else "lut_fast_kernel"


def per_dispatch(path, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if sub in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


f = per_dispatch(fcsv, "FETCH_SIZE")
w = per_dispatch(wcsv, "WRITE_SIZE")
if not f or not w:
    raise SystemExit(f"no {sub} dispatches in {fcsv} / {wcsv}")
fb = sum(f) / len(f) * 1024
wb = sum(w) / len(w) * 1024
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = os.path.join(root, "profiles", "pmc_traffic.json")
rec = json.load(open(out)) if os.path.exists(out) else {}
rec[key] = fb + wb
rec[key + "__detail"] = {"fetch_bytes": fb, "write_bytes": wb, "dispatches": [len(f), len(w)],
                         "note": "raw FETCH_SIZE+WRITE_SIZE (KiB->B), per launch, uncalibrated access width"}
json.dump(rec, open(out, "w"), indent=1, sort_keys=True)
print(key, fb + wb)
