#!/usr/bin/env bash
# LDS bank-conflict pass (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, one --pmc run
# each) of one bench step per library variant and kind.
# usage (GPU box): TAG=r06e bash tools/pmc_bank.sh VARIANT... (tree = the in-tree libqpd.so)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-bank}
O=gpurun_out/pmc_$TAG
mkdir -p "$O"
for v in "$@"; do
  lib=build_variants/libqpd_$v.so
  [ "$v" = "tree" ] && lib=quantized_decoder_polar_codes_amd/libqpd.so
  for kind in ${KINDS:-SCL-LUT FastSCL-LUT}; do
    QPD_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES \
      -d "$O/${v}_$kind" -o p --output-format csv -- python3 bench.py --kind $kind --steps 1 --warmup 0 \
      --no-cpu-baseline --no-e2e --frames 262144 > "$O/${v}_$kind.log" 2>&1 || { echo "pmc $v $kind failed"; exit 1; }
    python3 - "$O/${v}_$kind" "$v $kind" <<'PY'
import csv, glob, sys, collections
agg = collections.Counter()
for p in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"]
        if "lut_fast_kernel<" not in k:
            continue
        args = k.split("lut_fast_kernel<", 1)[1].split(">", 1)[0].replace(" ", "").split(",")
        if len(args) >= 5 and args[4] == "true":  # the frozen-prefix stages
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
bc, ia = agg["SQ_LDS_BANK_CONFLICT"], agg["SQ_LDS_IDX_ACTIVE"]
print(f"{sys.argv[2]:28s} bank_conflict {bc:.4g} idx_active {ia:.4g} ratio {bc / max(ia, 1):.4f} lds_insts {agg['SQ_INSTS_LDS']:.4g}")
PY
  done
done
