#!/bin/bash
# Round 3 ai: stage-2 record address in the import op records (no plan fields in the decode
# loop) -- prefix / parity / stream-safety tests, one interleaved A/B round (two stages / stage 1
# only / HEAD build), then rocprofv3 kernel statistics + PMC passes of the SCL-LUT bench workload.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
show() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline',{}); print('$2', round(d['value']/1e6,2), r.get('kernel_ms'), r.get('prefix_kernel_ms'), d['config'].get('prefix_ops'))"; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_prefix.py tests/test_gpu_parity.py tests/test_gpu_stream_safety.py tests/test_gpu_schedule_modes.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/r03ai_parity.log 2>&1
rc=$?; tail -2 $O/r03ai_parity.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
timeout -k 10 300 python bench.py --kind SCL-LUT --no-cpu-baseline --no-e2e > $O/r03ai_two$r.log 2>&1 || exit $?
show $O/r03ai_two$r.log "SCL-LUT two-stage"
QPD_NO_PFX2=1 timeout -k 10 300 python bench.py --kind SCL-LUT --no-cpu-baseline --no-e2e > $O/r03ai_one$r.log 2>&1 || exit $?
show $O/r03ai_one$r.log "SCL-LUT stage-1"
done
QPD_LIB=build_variants/libqpd_head.so timeout -k 10 300 python bench.py --kind SCL-LUT --no-cpu-baseline --no-e2e > $O/r03ai_head.log 2>&1 || exit $?
show $O/r03ai_head.log "SCL-LUT head"
timeout -k 10 600 bash tools/profile_round.sh r03ai_scl --kind SCL-LUT > $O/r03ai_prof_scl.log 2>&1 || exit $?
echo "profile done"
