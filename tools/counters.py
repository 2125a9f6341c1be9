"""Fold rocprofv3 PMC passes of one bench configuration into profiles/counters.json
(read by bench.py for `roofline.traffic` and `roofline.lds_hit`).

usage: python tools/counters.py KEY FRAMES PASS_CSV [PASS_CSV ...]

KEY is bench.py's record key (KIND_N.._K.._L.._F<frames per launch>); FRAMES
the frames one decode launch processes.  Each PASS_CSV is a
`*_counter_collection.csv` of one separate `rocprofv3 --pmc` pass
(tools/profile_round.sh: FETCH_SIZE; WRITE_SIZE; the SQ instruction mix; the
SQ wait/LDS counters).  Per kernel and per launch it records:

* fetch_raw / write: FETCH_SIZE and WRITE_SIZE in bytes (rocprofv3 reports KiB).
* fetch: fetch_raw x 2 -- MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE counts
  128-B memory-side requests at 64 B.  Calibrated here on root_pre_kernel,
  whose reads are exactly the 4 096 B of int32 channel symbols per frame
  (`pre_calibration` below: corrected fetch / algorithmic bytes).
* traffic = fetch + write (HBM-side bytes, Infinity-Cache hits included).
* lds_hit = SQ_INSTS_LDS / (SQ_INSTS_LDS + SQ_INSTS_VMEM_RD + SQ_INSTS_VMEM_WR):
  the fraction of the kernel's vector data-access instructions served by the
  LDS (ds_bpermute table lookups and fork copies, ds_read/ds_write of the
  LDS-resident tree rows) rather than by the vector-memory path (L1/L2/HBM:
  channel rows, table and quanta fetches, the global slab of the shallow tree
  depths, outputs).  SURVEY.md §8(d)'s "LDS-hit fraction".
* lds_bytes_hit: the same split weighted by bytes per wave-instruction
  (256 B for an LDS dword op; VMEM bytes = the TCP requests actually made,
  TCP_TOTAL_CACHE_ACCESSES x 64 B when that counter was collected).
"""
import collections
import csv
import json
import os
import sys

key, frames = sys.argv[1], float(sys.argv[2])
paths = [p for p in sys.argv[3:] if os.path.exists(p)]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
short = {"lut_fast_kernel": "lut_fast_kernel", "root_pre_kernel": "root_pre_kernel",
         "generic_decode_kernel": "generic_decode_kernel", "mc_frames_kernel": "mc_frames_kernel"}
def kernel_of(full):
    # lut_fast_kernel<KIND, NS, L8, R1L, PFX[, PW1]>: PFX true = the frozen-prefix stages
    if "lut_fast_kernel<" in full:
        args = full.split("lut_fast_kernel<", 1)[1].split(">", 1)[0].replace(" ", "").split(",")
        if len(args) >= 5 and args[4] == "true":
            return "lut_prefix_kernel"
    return next((s for s in short if s in full), None)


for p in paths:
    for r in csv.DictReader(open(p)):
        name = kernel_of(r["Kernel_Name"])
        if name is None:
            continue
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name][r["Counter_Name"]].add(r["Dispatch_Id"])

out = {"frames_per_launch": frames, "sources": [os.path.relpath(p) for p in paths], "kernels": {}}
for k, cs in agg.items():
    per = {c: v / max(1, len(disp[k][c])) for c, v in cs.items()}
    rec = {"per_launch": per, "per_frame": {c: v / frames for c, v in per.items()}}
    if "FETCH_SIZE" in per:
        rec["fetch_raw"] = per["FETCH_SIZE"] * 1024
        rec["fetch"] = 2 * rec["fetch_raw"]
    if "WRITE_SIZE" in per:
        rec["write"] = per["WRITE_SIZE"] * 1024
    if "fetch" in rec and "write" in rec:
        rec["traffic"] = rec["fetch"] + rec["write"]
    lds, rd, wr = per.get("SQ_INSTS_LDS"), per.get("SQ_INSTS_VMEM_RD"), per.get("SQ_INSTS_VMEM_WR")
    if lds is not None and rd is not None and wr is not None:
        rec["lds_hit"] = lds / (lds + rd + wr)
        tcp = per.get("TCP_TOTAL_CACHE_ACCESSES_sum")
        if tcp:
            rec["lds_bytes_hit"] = lds * 256 / (lds * 256 + tcp * 64)
    out["kernels"][k] = rec
pre = out["kernels"].get("root_pre_kernel", {})
if "fetch" in pre:
    n = int(key.split("_N")[1].split("_")[0])
    out["pre_calibration"] = pre["fetch"] / (frames * n * 4)

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(root, "profiles", "counters.json")
db = json.load(open(dst)) if os.path.exists(dst) else {}
db[key] = out
json.dump(db, open(dst, "w"), indent=1, sort_keys=True)
for k, rec in out["kernels"].items():
    print(k, {x: rec[x] for x in ("traffic", "lds_hit", "lds_bytes_hit") if x in rec})
if "pre_calibration" in out:
    print("pre_calibration (corrected fetch / algorithmic input bytes):", round(out["pre_calibration"], 4))
