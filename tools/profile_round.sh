#!/usr/bin/env bash
# Profiles for the record (run on the GPU box from the repo root):
#   kernel trace + stats of the default bench command, then separate PMC passes
#   (FETCH_SIZE, WRITE_SIZE, SQ instruction mix, LDS) -- never combined with
#   trace domains.  Writes under gpurun_out/prof_<tag>/; copy summaries to profiles/.
set -euo pipefail
TAG=${1:-r01}
shift || true
ARGS=${*:-"--steps 3 --warmup 1 --no-cpu-baseline"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof_$TAG
mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python3 bench.py $ARGS > "$O/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch" -o fetch --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$O/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$O/write" -o write --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$O/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES -d "$O/sqa" -o sqa --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$O/sqa.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$O/sqb" -o sqb --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$O/sqb.log" 2>&1
python3 tools/summarize_pmc.py 262144 "$O/sqa/sqa_counter_collection.csv" "$O/sqb/sqb_counter_collection.csv" > "$O/sq_summary.txt"
echo "profile $TAG done"
