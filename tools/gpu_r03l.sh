#!/bin/bash
# Round 3 l: the round's measurement record on the current build -- rocprofv3
# kernel statistics + separate PMC passes for SCL-LUT and FastSCL-LUT
# (tools/profile_round.sh), the bench lines with the CPU baseline, and
# BASELINE config 5 (10^8-frame Monte-Carlo point, with and without the stop rule).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python bench.py > $O/r03l_bench.log 2>&1 || exit $?
grep '^{' $O/r03l_bench.log > $O/r03l_bench.jsonl
timeout -k 10 400 python bench.py --kind FastSCL-LUT > $O/r03l_bench_fscl.log 2>&1 || exit $?
grep '^{' $O/r03l_bench_fscl.log > $O/r03l_bench_fscl.jsonl
timeout -k 10 300 python bench.py --mc-frames 1e8 > $O/r03l_mc_1e8.log 2>&1 || exit $?
grep '^{' $O/r03l_mc_1e8.log > $O/r03l_mc_1e8.jsonl
timeout -k 10 300 python bench.py --mc-frames 1e8 --mc-stop 1000 > $O/r03l_mc_stop.log 2>&1 || exit $?
grep '^{' $O/r03l_mc_stop.log > $O/r03l_mc_stop.jsonl
echo "bench records done"
timeout -k 10 600 bash tools/profile_round.sh r03l_scl --kind SCL-LUT > $O/r03l_prof_scl.log 2>&1 || exit $?
timeout -k 10 600 bash tools/profile_round.sh r03l_fscl --kind FastSCL-LUT > $O/r03l_prof_fscl.log 2>&1 || exit $?
echo profiles done
# scalar-cache behaviour of the op-record loads (optional: counter names may differ)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_ICACHE_MISSES -d $O/r03l_sqc -o p --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $O/r03l_sqc.log 2>&1 || echo "sqc pass failed"
echo sqc done
