#!/usr/bin/env bash
# Profiles for the record (run on the GPU box from the repo root):
#   kernel trace + stats of the bench command, then separate PMC passes
#   (FETCH_SIZE; WRITE_SIZE; SQ instruction mix; SQ waits / LDS; TCP/TCC) --
#   never combined with trace domains -- folded by tools/counters.py into
#   profiles/counters.json (bench.py's roofline.traffic / lds_hit).
# usage: bash tools/profile_round.sh TAG [bench args...]
# Writes under gpurun_out/prof_<tag>/; copies the summaries to gpurun_out/profiles_<tag>/.
set -euo pipefail
TAG=${1:-r02}
shift || true
ARGS=${*:-"--kind SCL-LUT"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof_$TAG
P=gpurun_out/profiles_$TAG
mkdir -p "$O" "$P"
B1="--steps 1 --warmup 0 --no-cpu-baseline --no-e2e $ARGS"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline $ARGS > "$O/kt.log" 2>&1
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d "$O/$name" -o "$name" --output-format csv -- python3 bench.py $B1 > "$O/$name.log" 2>&1
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass sqa SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES
pass sqb SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum || echo "tcp pass failed (optional)"
FR=$(python3 - "$ARGS" <<'EOF'
import sys
sys.path.insert(0, ".")
import bench
a = bench.parse(sys.argv[1].split())
print(f"{a.kind}_N{a.N}_K{a.K}_L{a.L}_F{a.frames} {a.frames}")
EOF
)
python3 tools/counters.py $FR "$O"/fetch/fetch_counter_collection.csv "$O"/write/write_counter_collection.csv \
  "$O"/sqa/sqa_counter_collection.csv "$O"/sqb/sqb_counter_collection.csv "$O"/tcp/tcp_counter_collection.csv \
  > "$P/counters_summary.txt"
cp profiles/counters.json "$P/counters.json"
cp "$O"/kt/kt_kernel_stats.csv "$P/kernel_stats.csv"
grep '^{' "$O/kt.log" | tail -1 > "$P/bench_under_rocprof.jsonl" || true
echo "profile $TAG done"
