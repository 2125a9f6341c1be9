#!/bin/bash
# Round 3 af: records on the current build (frozen-prefix stages) -- GPU suite, smoke,
# bench lines with the CPU baseline (SCL-LUT, FastSCL-LUT), the 10^8-frame Monte-Carlo
# point, per-frame latency.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/r03af_pytest_gpu.log 2>&1
rc=$?; tail -3 $O/r03af_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r03af_smoke.log 2>&1 || exit $?
tail -1 $O/r03af_smoke.log
timeout -k 10 400 python bench.py > $O/r03af_bench.log 2>&1 || exit $?
grep '^{' $O/r03af_bench.log > $O/r03af_bench.jsonl
timeout -k 10 400 python bench.py --kind FastSCL-LUT > $O/r03af_bench_fscl.log 2>&1 || exit $?
grep '^{' $O/r03af_bench_fscl.log > $O/r03af_bench_fscl.jsonl
timeout -k 10 300 python bench.py --mc-frames 1e8 > $O/r03af_mc_1e8.log 2>&1 || exit $?
grep '^{' $O/r03af_mc_1e8.log > $O/r03af_mc_1e8.jsonl
timeout -k 10 300 python tools/latency.py > $O/r03af_latency.jsonl 2> $O/r03af_latency.err || exit $?
echo "records done"
