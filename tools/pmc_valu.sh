#!/bin/bash
# The decode kernel's instruction mix on the bench workload (two separate
# rocprofv3 --pmc passes: SQ instruction counts; SQ waits / LDS / GRBM), then
# VALU instructions per frame and the VALU issue share (bench.py valu_ceiling).
# Run on the GPU box from the repo root.  usage: bash tools/pmc_valu.sh TAG [bench args...]
set -u
TAG=${1:-pmc}
shift || true
ARGS=${*:-"--kind SCL-LUT"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
B1="--steps 1 --warmup 0 --no-cpu-baseline --no-e2e $ARGS"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD \
  SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES -d "$O/sqa" -o sqa --output-format csv -- python3 bench.py $B1 > "$O/sqa.log" 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
  SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$O/sqb" -o sqb --output-format csv -- python3 bench.py $B1 > "$O/sqb.log" 2>&1 || exit $?
python3 - "$O" $ARGS <<'EOF'
import collections, csv, sys
sys.path.insert(0, ".")
import bench
o = sys.argv[1]
a = bench.parse(sys.argv[2:])
agg, disp = collections.defaultdict(float), collections.defaultdict(set)
for p in (f"{o}/sqa/sqa_counter_collection.csv", f"{o}/sqb/sqb_counter_collection.csv"):
    for r in csv.DictReader(open(p)):
        n = r["Kernel_Name"]
        if "lut_fast_kernel<" in n and n.split("lut_fast_kernel<", 1)[1].split(",")[4].strip() == "false":
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r["Dispatch_Id"])
per = {k: v / len(disp[k]) for k, v in agg.items()}
F = a.frames
print(f"{a.kind} frames/launch {F}: VALU/frame {per['SQ_INSTS_VALU'] / F:.0f}, SALU/frame {per['SQ_INSTS_SALU'] / F:.0f}, "
      f"LDS/frame {per['SQ_INSTS_LDS'] / F:.0f}, VALU issue share "
      f"{per['SQ_INSTS_VALU'] * bench.VALU_ISSUE_CYCLES / (bench.SIMDS * per['GRBM_GUI_ACTIVE'] / bench.XCDS):.3f}, "
      f"LDS bank conflicts {per['SQ_LDS_BANK_CONFLICT'] / per['SQ_LDS_IDX_ACTIVE']:.3f}")
EOF
