#!/bin/bash
# Instruction-fetch counters of the decode kernel (separate single-block passes).
# usage (GPU box, repo root): bash tools/pmc_icache.sh TAG [bench args...]
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
O=gpurun_out/ic_$TAG
mkdir -p $O
B="--steps 1 --warmup 0 --no-cpu-baseline --no-e2e $*"
for c in SQC_ICACHE_MISSES SQC_ICACHE_HITS "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $c -d $O/$n -o $n --output-format csv -- python3 bench.py $B > $O/$n.log 2>&1 || echo "pass $n failed"
done
python3 tools/counters.py ICACHE_$TAG 262144 $O/*/*_counter_collection.csv | grep lut_fast
python3 - $O <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(float); disp = collections.defaultdict(set)
for p in glob.glob(sys.argv[1] + "/*/*_counter_collection.csv"):
    for r in csv.DictReader(open(p)):
        if "lut_fast_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"]); disp[r["Counter_Name"]].add(r["Dispatch_Id"])
for k in sorted(agg):
    print(f"{k:28s} {agg[k] / max(1, len(disp[k])):18.0f}  per frame {agg[k] / max(1, len(disp[k])) / 262144:10.2f}")
PY
