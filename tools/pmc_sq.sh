#!/usr/bin/env bash
# SQ instruction-mix / stall / LDS counter passes (one --pmc set per run, no
# trace domains) of one bench step.  usage (GPU box): tools/pmc_sq.sh TAG [bench args]
set -euo pipefail
TAG=${1:-sq}
shift || true
ARGS=${*:-"--steps 1 --warmup 0 --no-cpu-baseline"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmc_$TAG
mkdir -p "$O"
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d "$O/p$i" -o p$i --output-format csv -- python3 bench.py $ARGS > "$O/p$i.log" 2>&1
done
python3 tools/summarize_pmc.py 262144 $(find "$O" -name "*counter_collection.csv" | sort) > "$O/summary.txt"
cat "$O/summary.txt"
