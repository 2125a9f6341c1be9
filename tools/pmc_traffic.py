"""Fold rocprofv3 FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_traffic.json
(HBM-side bytes per launch of the decode kernel), keyed like bench.py's lookup.

usage: python tools/pmc_traffic.py KEY FETCH_CSV WRITE_CSV [KERNEL_SUBSTR[,KERNEL_SUBSTR...]]
With several kernels (the root pre-pass + the decode kernel of one decode
call), their bytes are summed and divided by the first kernel's dispatches.
FETCH_SIZE/WRITE_SIZE are in KiB per dispatch (memory-side L2 requests; the
Infinity Cache is counted, not excluded -- MI355X_MICROARCH.md §HBM).  Our
reads are not 16-B/lane streaming loads, so the x2 FETCH correction for that
pattern does not apply; the value is reported raw and marked uncalibrated."""
import csv
import json
import os
import sys

key, fcsv, wcsv = sys.argv[1:4]
subs = (sys.argv[4] if len(sys.argv) > 4 else "lut_fast_kernel").split(",")


def per_call(path, counter):
    """Bytes per decode call: all matching kernels' counter sum / dispatches of subs[0]."""
    vals, first = 0.0, set()
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or not any(s in r["Kernel_Name"] for s in subs):
            continue
        vals += float(r["Counter_Value"])
        if subs[0] in r["Kernel_Name"]:
            first.add(r["Dispatch_Id"])
    return vals, len(first)


fv, fn = per_call(fcsv, "FETCH_SIZE")
wv, wn = per_call(wcsv, "WRITE_SIZE")
if not fn or not wn:
    raise SystemExit(f"no {subs[0]} dispatches in {fcsv} / {wcsv}")
f, w = [fv], [wv]
fb = fv / fn * 1024
wb = wv / wn * 1024
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = os.path.join(root, "profiles", "pmc_traffic.json")
rec = json.load(open(out)) if os.path.exists(out) else {}
rec[key] = fb + wb
rec[key + "__detail"] = {"fetch_bytes": fb, "write_bytes": wb, "dispatches": [fn, wn], "kernels": subs,
                         "note": "raw FETCH_SIZE+WRITE_SIZE (KiB->B), per launch, uncalibrated access width"}
json.dump(rec, open(out, "w"), indent=1, sort_keys=True)
print(key, fb + wb)
