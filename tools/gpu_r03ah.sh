#!/bin/bash
# Round 3 ah: two frozen-prefix stages for SCL-LUT -- the whole GPU suite, one interleaved
# A/B round (two stages / stage 1 only (QPD_NO_PFX2=1) / HEAD build), then the records of
# this build (smoke, bench lines with the CPU baseline, 10^8-frame Monte-Carlo point, latency).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
show() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline',{}); print('$2', round(d['value']/1e6,2), r.get('kernel_ms'), r.get('prefix_kernel_ms'), d['config'].get('prefix_ops'))"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r03ah_pytest_gpu.log 2>&1
rc=$?; tail -2 $O/r03ah_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --kind SCL-LUT --no-cpu-baseline --no-e2e > $O/r03ah_two.log 2>&1 || exit $?
show $O/r03ah_two.log "SCL-LUT two-stage"
QPD_NO_PFX2=1 timeout -k 10 300 python bench.py --kind SCL-LUT --no-cpu-baseline --no-e2e > $O/r03ah_one.log 2>&1 || exit $?
show $O/r03ah_one.log "SCL-LUT stage-1"
QPD_LIB=build_variants/libqpd_head.so timeout -k 10 300 python bench.py --kind SCL-LUT --no-cpu-baseline --no-e2e > $O/r03ah_head.log 2>&1 || exit $?
show $O/r03ah_head.log "SCL-LUT head"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r03ah_smoke.log 2>&1 || exit $?
tail -1 $O/r03ah_smoke.log
timeout -k 10 400 python bench.py > $O/r03ah_bench.log 2>&1 || exit $?
grep '^{' $O/r03ah_bench.log > $O/r03ah_bench.jsonl
show $O/r03ah_bench.log "bench"
timeout -k 10 400 python bench.py --kind FastSCL-LUT > $O/r03ah_bench_fscl.log 2>&1 || exit $?
grep '^{' $O/r03ah_bench_fscl.log > $O/r03ah_bench_fscl.jsonl
timeout -k 10 300 python bench.py --mc-frames 1e8 > $O/r03ah_mc_1e8.log 2>&1 || exit $?
grep '^{' $O/r03ah_mc_1e8.log > $O/r03ah_mc_1e8.jsonl
timeout -k 10 300 python tools/latency.py > $O/r03ah_latency.jsonl 2> $O/r03ah_latency.err || exit $?
echo "records done"
